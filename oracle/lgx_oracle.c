/*
 * lgx_oracle.c — CPU restatement of the legged_gym hot path.   TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline — never as the product path
 * (liblgx.so, HIP) and never as a fallback.
 *
 * What it restates (reference = /root/reference/legged_gym, cited file:line):
 *   - post_physics_step and everything it calls: legged_robot.py:109-231, 337-368,
 *     399-463, 818-966; isaacgym.torch_utils quaternion helpers as used there
 *     (quat_rotate_inverse / quat_apply, xyzw), utils/math.py:38-56.
 *     PINNED against golden vectors produced by the reference's own Python
 *     (tools/golden/gen_golden.py -> tests/golden/*.npz).
 *   - Go1 actuator-net history + UniNet MLP: envs/go1/go1.py:22-35,79-107 (pinned by the
 *     reference's go1_net.pt outputs), ANYmal SEA LSTM: envs/anymal_c/anymal.py:62-78
 *     (pinned by anydrive_v3_lstm.pt outputs).
 *   - the physics step that replaces Isaac Gym PhysX `gym.simulate` (closed source, absent):
 *     PARITY UNPINNED against PhysX.  The lgx physics model is restated here
 *     in a deliberately different formulation from the HIP kernel: dense 18x18 joint-space
 *     mass matrix H = sum_b J_b^T I_b J_b and dense Cholesky, vs the kernel's
 *     composite-rigid-body blocks + per-leg Schur complement; it is validated by
 *     known-answer physics tests (free fall, momentum, PD equilibrium) in tests/.
 *
 * Compiled with gcc -O2 -ffp-contract=off (oracle/Makefile).  Float32 arithmetic
 * throughout, like the reference (torch float32) and the kernel.
 */
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lgx.h"

#define ND 18 /* generalized velocity: [w(3), v(3), qd(12)] */

static float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

void lgxo_struct_sizes(int64_t out[3]) {
  out[0] = (int64_t)sizeof(lgx_model);
  out[1] = (int64_t)sizeof(lgx_env_params);
  out[2] = (int64_t)sizeof(lgx_buffers);
}

/* ------------------------------------------------------------------ Philox4x32-10 */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

/* uniform [0,1) for (env, slot) of draw stream `tag` at step `step` */
float lgxo_uniform(uint64_t seed, int32_t env, int32_t slot, int64_t step, uint32_t tag) {
  uint32_t c[4] = {(uint32_t)env, (uint32_t)(slot >> 2), (uint32_t)step, tag ^ ((uint32_t)((uint64_t)step >> 32) << 8)};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)(c[slot & 3] >> 8) * (1.0f / 16777216.0f);
}

typedef struct {
  const lgx_model* m;
  const lgx_env_params* p;
  const lgx_buffers* b;
  const float* draws; /* injected [N, stride] or NULL */
  int32_t stride;
  int32_t substep;    /* physics: substep index within the call (branch records) */
} ctx_t;

static float draw(const ctx_t* cx, int env, int slot, int64_t step, uint32_t tag) {
  if (cx->draws) return cx->draws[(int64_t)env * cx->stride + slot];
  return lgxo_uniform(cx->p->seed, env, slot, step, tag);
}

/* ------------------------------------------------------------------ arithmetic type of the physics
 * `real` is float (the product's arithmetic) unless built with -DLGXO_REAL=double: the float64
 * physics oracle (liblgx_oracle64.so, oracle/Makefile) that derives the physics tolerances - the
 * same algorithm in double precision, state read from / written to the float32 buffers at substep
 * boundaries (as in every build). */
#ifndef LGXO_REAL
#define LGXO_REAL float
#endif
typedef LGXO_REAL real;
#define LGXO_F64 (sizeof(real) == 8)
#define SQRT_R(x) (LGXO_F64 ? (real)sqrt(x) : (real)sqrtf(x))
#define FABS_R(x) (LGXO_F64 ? (real)fabs(x) : (real)fabsf(x))
#define FLOOR_R(x) (LGXO_F64 ? (real)floor(x) : (real)floorf(x))
#define FMAX_R(x, y) (LGXO_F64 ? (real)fmax(x, y) : (real)fmaxf(x, y))
#define FMIN_R(x, y) (LGXO_F64 ? (real)fmin(x, y) : (real)fminf(x, y))
#define COS_R(x) (LGXO_F64 ? (real)cos(x) : (real)cosf(x))
#define SIN_R(x) (LGXO_F64 ? (real)sin(x) : (real)sinf(x))
static void ldr(real* o, const float* s, int n) { for (int i = 0; i < n; ++i) o[i] = (real)s[i]; }

/* ------------------------------------------------------------------ small linear algebra */
static void cross3(const real* a, const real* b, real* o) {
  real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static real dot3(const real* a, const real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void matmul3(const real* A, const real* B, real* C) {
  real T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(C, T, sizeof T);
}
static void matvec3(const real* A, const real* x, real* y) {
  real t0 = A[0] * x[0] + A[1] * x[1] + A[2] * x[2];
  real t1 = A[3] * x[0] + A[4] * x[1] + A[5] * x[2];
  real t2 = A[6] * x[0] + A[7] * x[1] + A[8] * x[2];
  y[0] = t0; y[1] = t1; y[2] = t2;
}
static void quat_to_mat(const real* q, real* R) { /* xyzw */
  real x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}
static void axis_angle(const real* a, real th, real* R) { /* Rodrigues */
  real c = COS_R(th), s = SIN_R(th), t = 1 - c;
  real x = a[0], y = a[1], z = a[2];
  R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
  R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
  R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

/* isaacgym.torch_utils semantics (xyzw) */
static void quat_rotate_inverse(const real* q, const real* v, real* o) {
  real w = q[3];
  real a = 2.0f * w * w - 1.0f;
  real cx[3]; cross3(q, v, cx);
  real d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  for (int i = 0; i < 3; ++i) o[i] = v[i] * a - cx[i] * w * 2.0f + q[i] * d * 2.0f;
}
static void quat_apply(const real* q, const real* v, real* o) {
  real t[3]; cross3(q, v, t);
  for (int i = 0; i < 3; ++i) t[i] *= 2.0f;
  real u[3]; cross3(q, t, u);
  for (int i = 0; i < 3; ++i) o[i] = v[i] + q[3] * t[i] + u[i];
}

/* Cholesky solve of a dense SPD n x n system (in place, row-major lda = n) */
static void chol_solve(real* A, real* b, int n) {
  for (int j = 0; j < n; ++j) {
    real s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    real d = SQRT_R(s > 1e-20f ? s : 1e-20f);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      real t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  for (int i = 0; i < n; ++i) {
    real t = b[i];
    for (int k = 0; k < i; ++k) t -= A[i * n + k] * b[k];
    b[i] = t / A[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    real t = b[i];
    for (int k = i + 1; k < n; ++k) t -= A[k * n + i] * b[k];
    b[i] = t / A[i * n + i];
  }
}

/* ------------------------------------------------------------------ terrain */
/* ground height / normal of the triangulated heightfield (two triangles per cell, diagonal
 * (i,j)-(i+1,j+1), as isaacgym terrain_utils.convert_heightfield_to_trimesh builds it) */
static real ground(const ctx_t* cx, real x, real y, real* n) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  if (p->terrain_kind == 0 || !b->height_samples) { n[0] = 0; n[1] = 0; n[2] = 1; return 0.0f; }
  real ihs = 1.0f / p->horizontal_scale, vs = p->vertical_scale;   /* reciprocal scale, as the kernel */
  real u = (x + p->border_size) * ihs, v = (y + p->border_size) * ihs;
  int i = (int)FLOOR_R(u), j = (int)FLOOR_R(v);
  if (i < 0) i = 0; if (i > b->hf_rows - 2) i = b->hf_rows - 2;
  if (j < 0) j = 0; if (j > b->hf_cols - 2) j = b->hf_cols - 2;
  real fu = u - (real)i, fv = v - (real)j;
  if (fu < 0) fu = 0; if (fu > 1) fu = 1; if (fv < 0) fv = 0; if (fv > 1) fv = 1;
  const int16_t* H = b->height_samples;
  real h00 = H[i * b->hf_cols + j] * vs, h10 = H[(i + 1) * b->hf_cols + j] * vs;
  real h01 = H[i * b->hf_cols + j + 1] * vs, h11 = H[(i + 1) * b->hf_cols + j + 1] * vs;
  real gx, gy, h;
  if (fu >= fv) { gx = (h10 - h00) * ihs; gy = (h11 - h10) * ihs; h = h00 + fu * (h10 - h00) + fv * (h11 - h10); }
  else          { gx = (h11 - h01) * ihs; gy = (h01 - h00) * ihs; h = h00 + fv * (h01 - h00) + fu * (h11 - h01); }
  real inv = 1.0f / SQRT_R(gx * gx + gy * gy + 1.0f);
  n[0] = -gx * inv; n[1] = -gy * inv; n[2] = inv;
  return h;
}

/* ---- contact against the slope-corrected trimesh (terrain.py:70-73, legged_robot.py:629-643;
 * lgx_buffers.hf_trimesh): same model as the kernel, restated on plain arrays.  Closest point of a
 * triangle: Ericson, Real-Time Collision Detection 5.1.5. */
static void v3(real* o, real x, real y, real z) { o[0] = x; o[1] = y; o[2] = z; }
static void sub3(const real* a, const real* b, real* o) { v3(o, a[0] - b[0], a[1] - b[1], a[2] - b[2]); }
static void axpy3(const real* a, real s, const real* d, real* o) { v3(o, a[0] + s * d[0], a[1] + s * d[1], a[2] + s * d[2]); }

static void closest_on_tri(const real* p, const real* a, const real* b, const real* c, real* o) {
  real ab[3], ac[3], ap[3], bp[3], cq[3], bc[3];
  sub3(b, a, ab); sub3(c, a, ac); sub3(p, a, ap);
  real d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { memcpy(o, a, 3 * sizeof(real)); return; }
  sub3(p, b, bp);
  real d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { memcpy(o, b, 3 * sizeof(real)); return; }
  real vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { axpy3(a, d1 / (d1 - d3), ab, o); return; }
  sub3(p, c, cq);
  real d5 = dot3(ab, cq), d6 = dot3(ac, cq);
  if (d6 >= 0 && d5 <= d6) { memcpy(o, c, 3 * sizeof(real)); return; }
  real vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { axpy3(a, d2 / (d2 - d6), ac, o); return; }
  real va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    sub3(c, b, bc);
    axpy3(b, (d4 - d3) / ((d4 - d3) + (d5 - d6)), bc, o);
    return;
  }
  real den = 1.0f / (va + vb + vc);
  real t[3];
  axpy3(a, vb * den, ab, t);
  axpy3(t, vc * den, ac, o);
}

typedef struct { real d2, cp[3], cn[3], top, tn[3]; } tmq_t;

static void tm_tri(tmq_t* q, const real* p, const real* a, const real* b, const real* c) {
  real e1[3], e2[3], cp[3], dv[3];
  sub3(b, a, e1); sub3(c, a, e2);
  closest_on_tri(p, a, b, c, cp);
  sub3(p, cp, dv);
  real d2 = dot3(dv, dv);
  if (d2 < q->d2) { q->d2 = d2; memcpy(q->cp, cp, 3 * sizeof(real)); cross3(e1, e2, q->cn); }
  real den = e1[0] * e2[1] - e1[1] * e2[0];
  if (FABS_R(den) > 1e-9f) {
    real id = 1.0f / den;
    real px = p[0] - a[0], py = p[1] - a[1];
    real s = (px * e2[1] - py * e2[0]) * id, t = (e1[0] * py - e1[1] * px) * id;
    if (s >= -1e-6f && t >= -1e-6f && s + t <= 1.0f + 1e-6f) {
      real hz = a[2] + s * e1[2] + t * e2[2];
      if (hz > q->top) { q->top = hz; cross3(e1, e2, q->tn); }
    }
  }
}

/* signed depth of a sphere (radius r, centre p world) against the corrected mesh of the 3 x 3
 * cells around (i, j): nearest surface point, inside = below the surface under p */
static real trimesh_depth(const ctx_t* cx, const real* p, real r, int i, int j, real* n) {
  const lgx_env_params* P = cx->p;
  const lgx_buffers* b = cx->b;
  const real hs = P->horizontal_scale, vs = P->vertical_scale, bo = P->border_size;
  const int rows = b->hf_rows, cols = b->hf_cols;
  { /* early out: more than r above every vertex of the 4 x 4 block */
    int hmax = -32768;
    for (int a = i - 1; a <= i + 2; ++a)
      for (int bb = j - 1; bb <= j + 2; ++bb) {
        int aa = a < 0 ? 0 : (a > rows - 1 ? rows - 1 : a), bc = bb < 0 ? 0 : (bb > cols - 1 ? cols - 1 : bb);
        int h = b->height_samples[(int64_t)aa * cols + bc];
        if (h > hmax) hmax = h;
      }
    if (p[2] - r > (real)hmax * vs) { v3(n, 0, 0, 1); return -1.0f; }
  }
  /* frame at raw vertex (i, j): small coordinates (see the kernel) */
  const real ox = (real)i * hs - bo, oy = (real)j * hs - bo;
  real pl[3] = {p[0] - ox, p[1] - oy, p[2]};
  p = pl;
  tmq_t q;
  q.d2 = 3.0e38f; memcpy(q.cp, p, 3 * sizeof(real)); v3(q.cn, 0, 0, 1);
  q.top = -3.0e38f; v3(q.tn, 0, 0, 1);
  for (int ci = i - 1 < 0 ? 0 : i - 1; ci <= (i + 1 < rows - 2 ? i + 1 : rows - 2); ++ci)
    for (int cj = j - 1 < 0 ? 0 : j - 1; cj <= (j + 1 < cols - 2 ? j + 1 : cols - 2); ++cj) {
      real v[4][3];
      for (int k = 0; k < 4; ++k) {
        int a = ci + (k & 1), bb = cj + (k >> 1);
        int h = b->height_samples[(int64_t)a * cols + bb];
        int code = b->hf_trimesh[(int64_t)a * cols + bb] & 15;
        int dx = code / 3 - 1, dy = code % 3 - 1;
        v3(v[k], (real)(a + dx - i) * hs, (real)(bb + dy - j) * hs, (real)h * vs);
      }
      real zmax = v[0][2], xmin = v[0][0], xmax = v[0][0], ymin = v[0][1], ymax = v[0][1];
      for (int k = 1; k < 4; ++k) {
        zmax = FMAX_R(zmax, v[k][2]);
        xmin = FMIN_R(xmin, v[k][0]); xmax = FMAX_R(xmax, v[k][0]);
        ymin = FMIN_R(ymin, v[k][1]); ymax = FMAX_R(ymax, v[k][1]);
      }
      if (p[2] - r > zmax || p[0] < xmin - r || p[0] > xmax + r || p[1] < ymin - r || p[1] > ymax + r) continue;
      tm_tri(&q, p, v[0], v[3], v[2]);
      tm_tri(&q, p, v[0], v[1], v[3]);
    }
  int inside = p[2] < q.top;
  real d = SQRT_R(q.d2);
  if (d > 1e-7f) {
    real inv = 1.0f / d;
    for (int k = 0; k < 3; ++k) n[k] = inside ? inv * (q.cp[k] - p[k]) : inv * (p[k] - q.cp[k]);
  } else {
    const real* c = q.top > -1e30f ? q.tn : q.cn;
    real l = SQRT_R(dot3(c, c));
    real s = (c[2] < 0 ? -1.0f : 1.0f) / (l > 1e-30f ? l : 1e-30f);
    for (int k = 0; k < 3; ++k) n[k] = s * c[k];
  }
  return inside ? r + d : r - d;
}

/* ground contact depth of a sphere / point: spheres (r > 0) against the corrected trimesh where the
 * contact table flags the cell; box corners (r = 0) and unflagged cells against the heightfield
 * triangle under p, depth along its face normal (the kernel's split) */
static real ground_contact(const ctx_t* cx, const real* p, real r, real* n) {
  const lgx_env_params* P = cx->p;
  const lgx_buffers* b = cx->b;
  if (r > 0.0f && b->hf_trimesh && P->terrain_kind != 0 && b->height_samples) {
    const real ihs = 1.0f / P->horizontal_scale;
    int i = (int)FLOOR_R((p[0] + P->border_size) * ihs);
    int j = (int)FLOOR_R((p[1] + P->border_size) * ihs);
    if (i < 0) i = 0; if (i > b->hf_rows - 2) i = b->hf_rows - 2;
    if (j < 0) j = 0; if (j > b->hf_cols - 2) j = b->hf_cols - 2;
    if (b->hf_trimesh[(int64_t)i * b->hf_cols + j] & 16) return trimesh_depth(cx, p, r, i, j, n);
  }
  real h = ground(cx, p[0], p[1], n);
  return (h - p[2]) * n[2] + r;
}

/* test entry: ground_contact at world point p (radius r): depth, normal n[3] */
float lgxo_ground_contact(const lgx_env_params* p, const lgx_buffers* b, const float* pt, float r, float* n) {
  ctx_t cx = {NULL, p, b, NULL, 0};
  real ptr[3], nr[3];
  ldr(ptr, pt, 3);
  real d = ground_contact(&cx, ptr, (real)r, nr);
  for (int k = 0; k < 3; ++k) n[k] = (float)nr[k];
  return (float)d;
}

/* ------------------------------------------------------------------ physics substep */
typedef struct {
  real R[LGX_NUM_DYN][9];  /* body rotation (world) */
  real o[LGX_NUM_DYN][3];  /* body origin relative to base origin O */
  real S[LGX_NUM_DOF][6];  /* joint motion subspace (ang; lin) at O */
  real I6[LGX_NUM_DYN][36];
  int LD;                  /* joints per leg */
} kin_t;

/* legs of LD joints (lgx_model.leg_dof: 4 x 3 quadrupeds, 2 x 6 Cassie) */
static int leg_dof(const lgx_model* m) { return m->leg_dof == 6 ? 6 : 3; }
static int chain_has(int body, int joint, int LD) { /* does body's kinematic chain contain joint? */
  if (body == 0) return 0;
  int leg = (body - 1) / LD, k = (body - 1) % LD;
  return joint / LD == leg && joint % LD <= k;
}

static void spatial_inertia(const lgx_model* m, int b, real scale, const real* R, const real* o, real* I6) {
  const float* in = m->body_inertia[b];
  real Ib[9] = {in[0], in[3], in[4], in[3], in[1], in[5], in[4], in[5], in[2]};
  real T[9], RT[9], Iw[9];
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) RT[3 * i + j] = R[3 * j + i];
  matmul3(R, Ib, T); matmul3(T, RT, Iw);
  real com[3]; ldr(com, m->body_com[b], 3);
  real c[3]; matvec3(R, com, c);
  for (int i = 0; i < 3; ++i) c[i] += o[i];
  real mass = m->body_mass[b] * scale;
  for (int i = 0; i < 9; ++i) Iw[i] *= scale;
  real cc = dot3(c, c);
  memset(I6, 0, 36 * sizeof(real));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      I6[i * 6 + j] = Iw[3 * i + j] + mass * ((i == j ? cc : 0.0f) - c[i] * c[j]);
      I6[(3 + i) * 6 + 3 + j] = (i == j) ? mass : 0.0f;
    }
  real sk[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      I6[i * 6 + 3 + j] = mass * sk[3 * i + j];
      I6[(3 + i) * 6 + j] = mass * sk[3 * j + i];
    }
}

static void crm(const real* V, const real* s, real* o) { /* V x_m s */
  real a[3], l[3], t[3];
  cross3(V, s, a);
  cross3(V, s + 3, l); cross3(V + 3, s, t);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  o[3] = l[0] + t[0]; o[4] = l[1] + t[1]; o[5] = l[2] + t[2];
}
static void crf(const real* V, const real* f, real* o) { /* V x_f f */
  real a[3], b[3], l[3];
  cross3(V, f, a); cross3(V + 3, f + 3, b); cross3(V, f + 3, l);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  o[3] = l[0]; o[4] = l[1]; o[5] = l[2];
}
static void mv6(const real* M, const real* x, real* y) {
  for (int i = 0; i < 6; ++i) {
    real s = 0;
    for (int j = 0; j < 6; ++j) s += M[i * 6 + j] * x[j];
    y[i] = s;
  }
}

/* body Jacobian column of generalized coordinate c for body b (6-vector, ang;lin) */
static void body_jac_col(const kin_t* K, int b, int c, real* col) {
  memset(col, 0, 6 * sizeof(real));
  if (c < 6) { col[c] = 1.0f; return; }
  int j = c - 6;
  if (chain_has(b, j, K->LD)) memcpy(col, K->S[j], 6 * sizeof(real));
}

/* point Jacobian (3 x ND) of a point P (rel. O) on body b: v_P = v_lin + w x P */
static void point_jac(const kin_t* K, int b, const real* P, real* J) {
  memset(J, 0, 3 * ND * sizeof(real));
  for (int c = 0; c < ND; ++c) {
    real col[6]; body_jac_col(K, b, c, col);
    real wxp[3]; cross3(col, P, wxp);
    for (int r = 0; r < 3; ++r) J[r * ND + c] = col[3 + r] + wxp[r];
  }
}

typedef struct {
  int body, report;
  real J[3 * ND];
  real n[3];
  real depth;
  real mu;
  int status; /* 1 stick, 2 slide, 0 dropped */
  real fslide[3];
  int point;  /* candidate primitive (branch records) */
} contact_t;

static void add_weighted_jtj(real* A, const real* J, const real* n, real wn, real wt) {
  /* A += J^T (wn n n^T + wt (I - n n^T)) J */
  real W[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) W[3 * i + j] = (wn - wt) * n[i] * n[j] + (i == j ? wt : 0.0f);
  real WJ[3 * ND];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < ND; ++c) WJ[r * ND + c] = W[3 * r] * J[c] + W[3 * r + 1] * J[ND + c] + W[3 * r + 2] * J[2 * ND + c];
  for (int a = 0; a < ND; ++a)
    for (int c = 0; c < ND; ++c) A[a * ND + c] += J[a] * WJ[c] + J[ND + a] * WJ[ND + c] + J[2 * ND + a] * WJ[2 * ND + c];
}

#define MAXC LGX_MAX_POINTS

/* ---- branch records / forced branches of the physics (test infrastructure: the derived physics
 * tolerances of tests/test_gpu_parity.py).  The lgx contact model is discontinuous: every decision
 * below is identified by (env, substep of the lgxo_simulate call, kind, index) and recorded with
 * its decision and a relative margin to its threshold (|margin| small = within rounding of a
 * flip); a forced list makes the physics take the given decision instead of the computed one, so a
 * float64 run can follow the branch a float32 run took.
 *   kind 1  drive of joint `index`: 1 implicit PD drive (|te| <= effort), 0 saturated;
 *           margin (|te| - effort) / effort
 *   kind 2  limit of joint `index`: -1 below the lower limit, 0 inside, 1 above;
 *           margin = distance to the nearer limit (rad), negative outside
 *   kind 3  candidate primitive `index` in contact: 1 if depth > 0; margin depth / max(radius, 1 cm)
 *   kind 4  status of the contact of primitive `index` after pass 0: 0 separate (fn <= 0),
 *           1 stick, 2 slide (ct |vt| > mu fn); margin = the nearer of fn / (kn depth) and
 *           (ct |vt| - mu fn) / (mu fn) */
typedef struct {
  int32_t env, substep, kind, index, decision;
  float margin;
} lgxo_branch;
static lgxo_branch* g_rec;
static int64_t g_rec_cap, g_rec_n;
static const lgxo_branch* g_force;
static int64_t g_force_n;

void lgxo_branch_trace(lgxo_branch* buf, int64_t cap) {
  g_rec = buf;
  g_rec_cap = buf ? cap : 0;
  g_rec_n = 0;
}
int64_t lgxo_branch_count(void) { return g_rec_n; }
void lgxo_branch_force(const lgxo_branch* list, int64_t n) {
  g_force = list;
  g_force_n = list ? n : 0;
}

static int branch(const ctx_t* cx, int e, int kind, int index, int decision, real margin) {
  for (int64_t i = 0; i < g_force_n; ++i) {
    const lgxo_branch* f = &g_force[i];
    if (f->env == e && f->substep == cx->substep && f->kind == kind && f->index == index) {
      decision = f->decision;
      break;
    }
  }
  if (g_rec) {
    int64_t slot;
#pragma omp atomic capture
    slot = g_rec_n++;
    if (slot < g_rec_cap) {
      lgxo_branch r = {e, cx->substep, kind, index, decision, (float)margin};
      g_rec[slot] = r;
    }
  }
  return decision;
}

static void physics_env(const ctx_t* cx, int e) {
  const lgx_model* m = cx->m;
  const lgx_env_params* p = cx->p;
  const lgx_buffers* bf = cx->b;
  const real dt = m->sim_dt;
  float* rs = bf->root_states + (int64_t)e * 13;
  float* ds = bf->dof_state + (int64_t)e * 24;
  const float* tgt = bf->dof_targets + (int64_t)e * 12;
  real th[12], thd[12];
  for (int j = 0; j < 12; ++j) { th[j] = ds[2 * j]; thd[j] = ds[2 * j + 1]; }
  real u[ND];
  u[0] = rs[10]; u[1] = rs[11]; u[2] = rs[12]; u[3] = rs[7]; u[4] = rs[8]; u[5] = rs[9];
  for (int j = 0; j < 12; ++j) u[6 + j] = thd[j];

  /* kinematics */
  kin_t K;
  const int LD = leg_dof(m);
  K.LD = LD;
  real q0[4]; ldr(q0, rs + 3, 4);
  quat_to_mat(q0, K.R[0]);
  memset(K.o[0], 0, sizeof K.o[0]);
  for (int leg = 0; leg < LGX_NUM_DOF / LD; ++leg) {
    int pb = 0;
    for (int k = 0; k < LD; ++k) {
      int j = LD * leg + k, b = 1 + j;
      real Rjf[9], tmp[3], jrot[9], jpos[3], jax[3];
      ldr(jrot, m->joint_rot[j], 9); ldr(jpos, m->joint_pos[j], 3); ldr(jax, m->joint_axis[j], 3);
      matmul3(K.R[pb], jrot, Rjf);
      matvec3(K.R[pb], jpos, tmp);
      for (int i = 0; i < 3; ++i) K.o[b][i] = K.o[pb][i] + tmp[i];
      real aw[3]; matvec3(Rjf, jax, aw);
      real Rq[9]; axis_angle(jax, th[j], Rq);
      matmul3(Rjf, Rq, K.R[b]);
      K.S[j][0] = aw[0]; K.S[j][1] = aw[1]; K.S[j][2] = aw[2];
      cross3(K.o[b], aw, K.S[j] + 3);
      pb = b;
    }
  }
  const float* mscale = bf->body_mass_scale + (int64_t)e * LGX_NUM_DYN;
  for (int b = 0; b < LGX_NUM_DYN; ++b) spatial_inertia(m, b, mscale[b], K.R[b], K.o[b], K.I6[b]);

  /* mass matrix H = sum_b J_b^T I_b J_b (dense) */
  real H[ND * ND];
  memset(H, 0, sizeof H);
  for (int b = 0; b < LGX_NUM_DYN; ++b) {
    real Jb[6 * ND];
    for (int c = 0; c < ND; ++c) {
      real col[6]; body_jac_col(&K, b, c, col);
      for (int r = 0; r < 6; ++r) Jb[r * ND + c] = col[r];
    }
    real IJ[6 * ND];
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < ND; ++c) {
        real s = 0;
        for (int k = 0; k < 6; ++k) s += K.I6[b][r * 6 + k] * Jb[k * ND + c];
        IJ[r * ND + c] = s;
      }
    for (int a = 0; a < ND; ++a)
      for (int c = 0; c < ND; ++c) {
        real s = 0;
        for (int k = 0; k < 6; ++k) s += Jb[k * ND + a] * IJ[k * ND + c];
        H[a * ND + c] += s;
      }
  }

  /* bias forces C = sum_b J_b^T (I_b A_b + V_b x* I_b V_b), A_0 = (0, -w x v - g) */
  real V[LGX_NUM_DYN][6], A[LGX_NUM_DYN][6];
  memcpy(V[0], u, 6 * sizeof(real));
  real wxv[3]; cross3(u, u + 3, wxv);
  A[0][0] = A[0][1] = A[0][2] = 0;
  for (int i = 0; i < 3; ++i) A[0][3 + i] = -wxv[i] - m->gravity[i];
  for (int leg = 0; leg < LGX_NUM_DOF / LD; ++leg) {
    int pb = 0;
    for (int k = 0; k < LD; ++k) {
      int j = LD * leg + k, b = 1 + j;
      for (int i = 0; i < 6; ++i) V[b][i] = V[pb][i] + K.S[j][i] * thd[j];
      real c6[6]; crm(V[b], K.S[j], c6);
      for (int i = 0; i < 6; ++i) A[b][i] = A[pb][i] + c6[i] * thd[j];
      pb = b;
    }
  }
  real Cb[ND];
  memset(Cb, 0, sizeof Cb);
  for (int b = 0; b < LGX_NUM_DYN; ++b) {
    real IA[6], IV[6], f[6], vf[6];
    mv6(K.I6[b], A[b], IA); mv6(K.I6[b], V[b], IV); crf(V[b], IV, vf);
    for (int i = 0; i < 6; ++i) f[i] = IA[i] + vf[i];
    for (int c = 0; c < ND; ++c) {
      real col[6]; body_jac_col(&K, b, c, col);
      real s = 0;
      for (int i = 0; i < 6; ++i) s += col[i] * f[i];
      Cb[c] += s;
    }
  }

  /* joint drives / explicit torques, hard limits */
  real g[ND]; memset(g, 0, sizeof g);
  real Dimp[12]; int implicit_drive[12];
  for (int j = 0; j < 12; ++j) {
    Dimp[j] = 0; implicit_drive[j] = 0;
    real eff = m->dof_effort[j];
    if (p->control_type == LGX_CTRL_POS_DRIVE) {
      real te = m->kp[j] * (tgt[j] - th[j]) - m->kd[j] * thd[j];
      if (branch(cx, e, 1, j, FABS_R(te) <= eff, (FABS_R(te) - eff) / eff)) {
        implicit_drive[j] = 1;
        Dimp[j] += dt * (m->kd[j] + dt * m->kp[j]);
        g[6 + j] += m->kp[j] * (tgt[j] - th[j]);
      } else {
        g[6 + j] += te > 0 ? eff : -eff;
      }
    } else {
      g[6 + j] += bf->torques[(int64_t)e * 12 + j]; /* explicit torques precomputed by caller */
    }
    if (m->dof_lower[j] < m->dof_upper[j]) {
      const int lim = branch(cx, e, 2, j, th[j] < m->dof_lower[j] ? -1 : (th[j] > m->dof_upper[j] ? 1 : 0),
                             FMIN_R(th[j] - m->dof_lower[j], m->dof_upper[j] - th[j]));
      if (lim < 0) {
        Dimp[j] += dt * (m->limit_c + dt * m->limit_k);
        g[6 + j] += m->limit_k * (m->dof_lower[j] - th[j]);
      } else if (lim > 0) {
        Dimp[j] += dt * (m->limit_c + dt * m->limit_k);
        g[6 + j] -= m->limit_k * (th[j] - m->dof_upper[j]);
      }
    }
  }

  /* contacts (candidates = every primitive below the ground) */
  contact_t C[MAXC];
  int nc = 0;
  real mu_env = bf->friction ? bf->friction[e] : 1.0f;
  for (int i = 0; i < m->num_points; ++i) {
    int b = m->point_dyn[i];
    real ppos[3]; ldr(ppos, m->point_pos[i], 3);
    real P[3]; matvec3(K.R[b], ppos, P);
    for (int k = 0; k < 3; ++k) P[k] += K.o[b][k];
    real n[3];
    const real Pw[3] = {P[0] + rs[0], P[1] + rs[1], P[2] + rs[2]};
    real depth = ground_contact(cx, Pw, m->point_radius[i], n);
    if (!branch(cx, e, 3, i, depth > 0.0f, depth / FMAX_R((real)m->point_radius[i], (real)0.01f))) continue;
    contact_t* c = &C[nc++];
    c->point = i;
    c->body = b; c->report = m->point_report[i];
    real Pc[3] = {P[0] - n[0] * m->point_radius[i], P[1] - n[1] * m->point_radius[i], P[2] - n[2] * m->point_radius[i]};
    point_jac(&K, b, Pc, c->J);
    memcpy(c->n, n, sizeof n);
    c->depth = depth;
    c->mu = 0.5f * (mu_env + m->ground_friction);
    c->status = 1;
  }

  real Hu[ND];
  for (int a = 0; a < ND; ++a) {
    real s = 0;
    for (int c = 0; c < ND; ++c) s += H[a * ND + c] * u[c];
    Hu[a] = s;
  }
  const real kn = m->contact_k, cn = m->contact_c, ct = m->friction_c;
  real u2[ND];
  for (int pass = 0; pass < 2; ++pass) {
    real M[ND * ND], r[ND];
    memcpy(M, H, sizeof M);
    for (int j = 0; j < 12; ++j) M[(6 + j) * ND + 6 + j] += Dimp[j];
    for (int a = 0; a < ND; ++a) r[a] = Hu[a] + dt * (g[a] - Cb[a]);
    for (int i = 0; i < nc; ++i) {
      contact_t* c = &C[i];
      if (c->status == 0) continue;
      real wt = (pass == 0 || c->status == 1) ? dt * ct : 0.0f;
      add_weighted_jtj(M, c->J, c->n, dt * (cn + dt * kn), wt);
      for (int a = 0; a < ND; ++a) {
        real jn = c->J[a] * c->n[0] + c->J[ND + a] * c->n[1] + c->J[2 * ND + a] * c->n[2];
        r[a] += dt * kn * c->depth * jn;
        if (pass == 1 && c->status == 2)
          r[a] += dt * (c->J[a] * c->fslide[0] + c->J[ND + a] * c->fslide[1] + c->J[2 * ND + a] * c->fslide[2]);
      }
    }
    chol_solve(M, r, ND);
    memcpy(u2, r, sizeof u2);
    if (pass == 0) {
      for (int i = 0; i < nc; ++i) {
        contact_t* c = &C[i];
        real vp[3];
        for (int k = 0; k < 3; ++k) {
          real s = 0;
          for (int a = 0; a < ND; ++a) s += c->J[k * ND + a] * u2[a];
          vp[k] = s;
        }
        real vn = dot3(vp, c->n);
        real fn = kn * c->depth - (cn + dt * kn) * vn;
        real vt[3] = {vp[0] - vn * c->n[0], vp[1] - vn * c->n[1], vp[2] - vn * c->n[2]};
        real vtn = SQRT_R(dot3(vt, vt));
        const int st = fn <= 0.0f ? 0 : (ct * vtn > c->mu * fn ? 2 : 1);
        const real m_sep = fn / FMAX_R(kn * FABS_R(c->depth), (real)1e-6f);
        const real m_slide = (ct * vtn - c->mu * fn) / FMAX_R(c->mu * FABS_R(fn), (real)1e-6f);
        c->status = branch(cx, e, 4, c->point, st, FABS_R(m_sep) < FABS_R(m_slide) ? m_sep : m_slide);
        if (c->status == 2) {
          real s = -c->mu * fn / FMAX_R(vtn, (real)1e-12f);
          c->fslide[0] = s * vt[0]; c->fslide[1] = s * vt[1]; c->fslide[2] = s * vt[2];
        }
      }
    }
  }

  /* reported contact forces (last substep) */
  float* cf = bf->contact_forces + (int64_t)e * LGX_MAX_BODIES * 3;
  memset(cf, 0, (size_t)LGX_MAX_BODIES * 3 * sizeof(float));
  for (int i = 0; i < nc; ++i) {
    contact_t* c = &C[i];
    if (c->status == 0) continue;
    real vp[3];
    for (int k = 0; k < 3; ++k) {
      real s = 0;
      for (int a = 0; a < ND; ++a) s += c->J[k * ND + a] * u2[a];
      vp[k] = s;
    }
    real vn = dot3(vp, c->n);
    real fn = kn * c->depth - (cn + dt * kn) * vn;
    if (fn < 0) fn = 0;
    real f[3];
    for (int k = 0; k < 3; ++k) {
      real ft = c->status == 1 ? -ct * (vp[k] - vn * c->n[k]) : c->fslide[k];
      f[k] = fn * c->n[k] + ft;
    }
    for (int k = 0; k < 3; ++k) cf[c->report * 3 + k] += f[k];
  }

  /* joint outputs */
  float* tq = bf->torques + (int64_t)e * 12;
  for (int j = 0; j < 12; ++j) {
    real qd = u2[6 + j];
    real vl = m->dof_vel_limit[j];
    if (vl > 0) { if (qd > vl) qd = vl; if (qd < -vl) qd = -vl; }
    if (p->control_type == LGX_CTRL_POS_DRIVE) {
      real eff = m->dof_effort[j];
      real t;
      if (implicit_drive[j]) t = m->kp[j] * (tgt[j] - th[j] - dt * u2[6 + j]) - m->kd[j] * u2[6 + j];
      else t = m->kp[j] * (tgt[j] - th[j]) - m->kd[j] * thd[j];
      if (t > eff) t = eff; if (t < -eff) t = -eff;
      tq[j] = t;
    }
    ds[2 * j] = th[j] + dt * qd;
    ds[2 * j + 1] = qd;
  }
  /* root integration (semi-implicit Euler; quaternion q' = q + dt/2 (w,0) x q, normalised) */
  real w[3] = {u2[0], u2[1], u2[2]}, v[3] = {u2[3], u2[4], u2[5]};
  for (int i = 0; i < 3; ++i) rs[i] = (float)((real)rs[i] + dt * v[i]);
  real q[4]; ldr(q, rs + 3, 4);
  real wq[3]; cross3(w, q, wq);
  real dq[4] = {0.5f * (q[3] * w[0] + wq[0]), 0.5f * (q[3] * w[1] + wq[1]), 0.5f * (q[3] * w[2] + wq[2]),
                 -0.5f * dot3(w, q)};
  for (int i = 0; i < 4; ++i) q[i] += dt * dq[i];
  real qn = 1.0f / SQRT_R(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) rs[3 + i] = (float)(q[i] * qn);
  rs[7] = v[0]; rs[8] = v[1]; rs[9] = v[2];
  rs[10] = w[0]; rs[11] = w[1]; rs[12] = w[2];
}

#ifndef LGXO_PHYSICS_ONLY   /* (the float64 build holds the physics alone) */
/* ------------------------------------------------------------------ actuator history (Go1) */
static void actuator_history(const ctx_t* cx, int e, int substep) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  const float* a = b->actions + (int64_t)e * 12;
  const float* ds = b->dof_state + (int64_t)e * 24;
  float* h = b->act_hist + (int64_t)e * 120;  /* [12][2][5] */
  float* mi = b->model_ins + ((int64_t)substep * p->num_envs + e) * 120;
  for (int j = 0; j < 12; ++j) {
    float pe = a[j] - ds[2 * j];                                     /* go1.py:82 */
    float pes = (pe - p->act_pos_err_mean[j]) / p->act_pos_err_std[j];
    float vs = (ds[2 * j + 1] - p->act_vel_mean[j]) / p->act_vel_std[j];
    float* hp = h + j * 10;
    float* hv = hp + 5;
    for (int k = 0; k < 4; ++k) { hp[k] = hp[k + 1]; hv[k] = hv[k + 1]; }  /* np.delete + append */
    hp[4] = pes; hv[4] = vs;
    memcpy(mi + j * 10, hp, 10 * sizeof(float));                      /* go1.py:96-97 */
  }
}

/* one substep of the Go1 actuator history for all envs (replay of go1.py:79-98) */
void lgxo_actuator_history(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, int substep) {
  ctx_t cx = {m, p, b, NULL, 0};
  for (int e = 0; e < p->num_envs; ++e) actuator_history(&cx, e, substep);
}

/* ------------------------------------------------------------------ env step pieces */

void lgxo_compute_targets(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b) {
  (void)m;
  for (int e = 0; e < p->num_envs; ++e)
    for (int j = 0; j < 12; ++j) {  /* _compute_poses, legged_robot.py:394-397 */
      float t = b->actions[e * 12 + j] * p->action_scale + p->default_dof_pos[j];
      b->dof_targets[e * 12 + j] = clampf(t, p->soft_lower[j], p->soft_upper[j]);
    }
}

/* explicit-torque controllers, _compute_torques (legged_robot.py:370-392) */
void lgxo_explicit_torques(const lgx_env_params* p, const lgx_buffers* b) {
  for (int e = 0; e < p->num_envs; ++e)
    for (int j = 0; j < 12; ++j) {
      float a = b->actions[e * 12 + j] * p->action_scale;
      float q = b->dof_state[e * 24 + 2 * j], qd = b->dof_state[e * 24 + 2 * j + 1], t;
      if (p->control_type == LGX_CTRL_P) t = p->p_gains[j] * (a + p->default_dof_pos[j] - q) - p->d_gains[j] * qd;
      else if (p->control_type == LGX_CTRL_V)
        t = p->p_gains[j] * (a - qd) - p->d_gains[j] * (qd - b->last_dof_vel[e * 12 + j]) / (p->dt / (float)p->decimation);
      else t = a;
      b->torques[e * 12 + j] = clampf(t, -p->torque_limits[j], p->torque_limits[j]);
    }
}

#endif /* LGXO_PHYSICS_ONLY */

void lgxo_simulate(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, int n) {
  ctx_t cx = {m, p, b, NULL, 0, 0};
  for (int s = 0; s < n; ++s) {
    cx.substep = s;
    for (int e = 0; e < p->num_envs; ++e) physics_env(&cx, e);
  }
}

#ifndef LGXO_PHYSICS_ONLY
static void resample_cmd(const ctx_t* cx, int e, int slot, int64_t step, uint32_t tag) {
  const lgx_env_params* p = cx->p;
  float* c = cx->b->commands + (int64_t)e * 4;
  for (int k = 0; k < 2; ++k) {
    float lo = p->cmd_ranges[k][0], hi = p->cmd_ranges[k][1];
    c[k] = (hi - lo) * draw(cx, e, slot + k, step, tag) + lo;
  }
  int k3 = p->heading_command ? 3 : 2;
  float lo = p->cmd_ranges[k3][0], hi = p->cmd_ranges[k3][1];
  c[k3] = (hi - lo) * draw(cx, e, slot + 2, step, tag) + lo;
  float nrm = sqrtf(c[0] * c[0] + c[1] * c[1]);
  float keep = nrm > 0.2f ? 1.0f : 0.0f;
  c[0] *= keep; c[1] *= keep;
}

static float wrap_to_pi(float a) {
  const float tp = (float)(2.0 * 3.14159265358979323846);
  float r = fmodf(a, tp);
  if (r != 0.0f && r < 0.0f) r += tp;
  if (r > (float)3.14159265358979323846) r -= tp;
  return r;
}

static void get_heights(const ctx_t* cx, int e) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  float* mh = b->measured_heights + (int64_t)e * p->num_height_points;
  if (p->terrain_kind == 0) { for (int i = 0; i < p->num_height_points; ++i) mh[i] = 0.0f; return; }
  const float* rs = b->root_states + (int64_t)e * 13;
  float qy[4] = {0, 0, rs[5], rs[6]};
  float nrm = sqrtf(qy[2] * qy[2] + qy[3] * qy[3]);
  if (nrm < 1e-9f) nrm = 1e-9f;
  qy[2] /= nrm; qy[3] /= nrm;
  for (int i = 0; i < p->num_height_points; ++i) {
    float v[3] = {p->height_points[i][0], p->height_points[i][1], 0.0f}, o[3];
    quat_apply(qy, v, o);
    float x = o[0] + rs[0] + p->border_size, y = o[1] + rs[1] + p->border_size;
    int64_t px = (int64_t)(x / p->horizontal_scale), py = (int64_t)(y / p->horizontal_scale);
    if (px < 0) px = 0; if (px > b->hf_rows - 2) px = b->hf_rows - 2;
    if (py < 0) py = 0; if (py > b->hf_cols - 2) py = b->hf_cols - 2;
    const int16_t* H = b->height_samples;
    int16_t h1 = H[px * b->hf_cols + py], h2 = H[(px + 1) * b->hf_cols + py], h3 = H[px * b->hf_cols + py + 1];
    int16_t h = h1 < h2 ? h1 : h2;
    h = h < h3 ? h : h3;
    mh[i] = (float)h * p->vertical_scale;
  }
}

static float norm3(const float* f) { return sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]); }

static float reward_term(const ctx_t* cx, int e, int id) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  const float* blv = b->base_lin_vel + e * 3;
  const float* bav = b->base_ang_vel + e * 3;
  const float* pg = b->projected_gravity + e * 3;
  const float* ds = b->dof_state + (int64_t)e * 24;
  const float* tq = b->torques + (int64_t)e * 12;
  const float* cf = b->contact_forces + (int64_t)e * LGX_MAX_BODIES * 3;
  const float* cmd = b->commands + e * 4;
  const float* act = b->actions + e * 12;
  const float* la = b->last_actions + e * 12;
  const float* ldv = b->last_dof_vel + e * 12;
  float s = 0.0f;
  switch (id) {
    case LGX_R_LIN_VEL_Z: return blv[2] * blv[2];
    case LGX_R_ANG_VEL_XY: return bav[0] * bav[0] + bav[1] * bav[1];
    case LGX_R_ORIENTATION: return pg[0] * pg[0] + pg[1] * pg[1];
    case LGX_R_BASE_HEIGHT: {
      float z = b->root_states[e * 13 + 2];
      float acc = 0;
      if (p->measure_heights) {
        for (int i = 0; i < p->num_height_points; ++i) acc += z - b->measured_heights[e * p->num_height_points + i];
        acc /= (float)p->num_height_points;
      } else acc = z;
      float d = acc - p->base_height_target;
      return d * d;
    }
    case LGX_R_TORQUES: for (int j = 0; j < 12; ++j) s += tq[j] * tq[j]; return s;
    case LGX_R_ENERGY: for (int j = 0; j < 12; ++j) { float x = tq[j] * ds[2 * j + 1]; s += x * x; } return s;
    case LGX_R_DOF_VEL: for (int j = 0; j < 12; ++j) s += ds[2 * j + 1] * ds[2 * j + 1]; return s;
    case LGX_R_DOF_ACC: for (int j = 0; j < 12; ++j) { float x = (ldv[j] - ds[2 * j + 1]) / p->dt; s += x * x; } return s;
    case LGX_R_ACTION_RATE: for (int j = 0; j < 12; ++j) { float x = la[j] - act[j]; s += x * x; } return s;
    case LGX_R_COLLISION:
      for (int i = 0; i < p->num_penalised; ++i) s += norm3(cf + 3 * p->penalised_indices[i]) > 0.1f ? 1.0f : 0.0f;
      return s;
    case LGX_R_TERMINATION: return (b->reset[e] && !b->time_out[e]) ? 1.0f : 0.0f;
    case LGX_R_DOF_POS_LIMITS:
      for (int j = 0; j < 12; ++j) {
        float lo = ds[2 * j] - p->soft_lower[j], hi = ds[2 * j] - p->soft_upper[j];
        s += -(lo < 0 ? lo : 0.0f) + (hi > 0 ? hi : 0.0f);
      }
      return s;
    case LGX_R_DOF_VEL_LIMITS:
      for (int j = 0; j < 12; ++j) s += clampf(fabsf(ds[2 * j + 1]) - p->dof_vel_limits[j] * p->soft_dof_vel_limit, 0.0f, 1.0f);
      return s;
    case LGX_R_TORQUE_LIMITS:
      for (int j = 0; j < 12; ++j) { float x = fabsf(tq[j]) - p->torque_limits[j] * p->soft_torque_limit; s += x > 0 ? x : 0.0f; }
      return s;
    case LGX_R_TRACKING_LIN_VEL: {
      float ex = cmd[0] - blv[0], ey = cmd[1] - blv[1];
      return expf(-(ex * ex + ey * ey) / p->tracking_sigma);
    }
    case LGX_R_TRACKING_ANG_VEL: { float ez = cmd[2] - bav[2]; return expf(-(ez * ez) / p->tracking_sigma); }
    case LGX_R_FEET_AIR_TIME: { /* mutates feet_air_time (legged_robot.py:941-949) */
      float* fat = b->feet_air_time + e * 4;
      for (int f = 0; f < p->num_feet; ++f) {
        int contact = cf[3 * p->feet_indices[f] + 2] > 1.0f;
        float first = (fat[f] > 0.0f && contact) ? 1.0f : 0.0f;
        fat[f] += p->dt;
        s += (fat[f] - 0.5f) * first;
      }
      s *= (sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) > 0.1f) ? 1.0f : 0.0f;
      for (int f = 0; f < p->num_feet; ++f) if (cf[3 * p->feet_indices[f] + 2] > 1.0f) fat[f] = 0.0f;
      return s;
    }
    case LGX_R_STUMBLE:
      for (int f = 0; f < p->num_feet; ++f) {
        const float* F = cf + 3 * p->feet_indices[f];
        if (sqrtf(F[0] * F[0] + F[1] * F[1]) > 5.0f * fabsf(F[2])) return 1.0f;
      }
      return 0.0f;
    case LGX_R_STAND_STILL:
      for (int j = 0; j < 12; ++j) s += fabsf(ds[2 * j] - p->default_dof_pos[j]);
      return s * ((sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) < 0.1f) ? 1.0f : 0.0f);
    case LGX_R_FEET_CONTACT_FORCES:
      for (int f = 0; f < p->num_feet; ++f) { float x = norm3(cf + 3 * p->feet_indices[f]) - p->max_contact_force; s += x > 0 ? x : 0.0f; }
      return s;
    case LGX_R_HIP_MOTION:
      for (int j = 0; j < 12; j += 3) s += fabsf(ds[2 * j] - p->default_dof_pos[j]);
      return s;
    case LGX_R_NO_FLY: { /* envs/cassie/cassie.py:42-46 */
      int n = 0;
      for (int f = 0; f < p->num_feet; ++f) n += cf[3 * p->feet_indices[f] + 2] > 0.1f;
      return n == 1 ? 1.0f : 0.0f;
    }
  }
  return 0.0f;
}

static int nterm_rows(const lgx_env_params* p) { return p->num_terms + (p->termination_slot >= 0 ? 1 : 0); }

/* reset_idx for a list of envs (legged_robot.py:150-193) */
static void reset_envs(const ctx_t* cx, const int32_t* ids, int n, int64_t step, uint32_t tag, int init_done) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  int N = p->num_envs;
  if (n == 0) return;
  if (p->curriculum && init_done) {  /* _update_terrain_curriculum :443-463 */
    for (int k = 0; k < n; ++k) {
      int e = ids[k];
      const float* rs = b->root_states + e * 13;
      float* org = b->env_origins + e * 3;
      float dx = rs[0] - org[0], dy = rs[1] - org[1];
      float dist = sqrtf(dx * dx + dy * dy);
      const float* c = b->commands + e * 4;
      int up = dist > p->terrain_env_length / 2.0f;
      int down = (dist < sqrtf(c[0] * c[0] + c[1] * c[1]) * p->max_episode_length_s * 0.5f) && !up;
      int64_t lvl = b->terrain_levels[e] + up - down;
      if (lvl >= p->max_terrain_level) {
        int64_t r = (int64_t)(draw(cx, e, LGX_DRAW_CURRIC, step, tag) * (float)p->max_terrain_level);
        if (r >= p->max_terrain_level) r = p->max_terrain_level - 1;
        lvl = r;
      } else if (lvl < 0) lvl = 0;
      b->terrain_levels[e] = lvl;
      const float* to = b->terrain_origins + (lvl * p->terrain_num_cols + b->terrain_types[e]) * 3;
      org[0] = to[0]; org[1] = to[1]; org[2] = to[2];
    }
  }
  for (int k = 0; k < n; ++k) {
    int e = ids[k];
    float* ds = b->dof_state + e * 24;
    for (int j = 0; j < 12; ++j) {
      ds[2 * j] = p->default_dof_pos[j] * ((1.5f - 0.5f) * draw(cx, e, LGX_DRAW_RESET_DOF + j, step, tag) + 0.5f);
      ds[2 * j + 1] = 0.0f;
    }
    float* rs = b->root_states + e * 13;
    for (int i = 0; i < 13; ++i) rs[i] = p->base_init_state[i];
    for (int i = 0; i < 3; ++i) rs[i] += b->env_origins[e * 3 + i];
    if (p->custom_origins)
      for (int i = 0; i < 2; ++i) rs[i] += (1.0f - -1.0f) * draw(cx, e, LGX_DRAW_RESET_XY + i, step, tag) + -1.0f;
    for (int i = 0; i < 6; ++i) rs[7 + i] = (0.5f - -0.5f) * draw(cx, e, LGX_DRAW_RESET_VEL + i, step, tag) + -0.5f;
    resample_cmd(cx, e, LGX_DRAW_RESET_CMD, step, tag);
    for (int j = 0; j < 12; ++j) { b->last_actions[e * 12 + j] = 0; b->last_dof_vel[e * 12 + j] = 0; }
    for (int f = 0; f < 4; ++f) b->feet_air_time[e * 4 + f] = 0;
    if (b->sea_h && b->sea_c) /* Anymal.reset_idx zeroes the SEA LSTM state (anymal.py:56-60) */
      for (int L = 0; L < 2; ++L) {
        memset(b->sea_h + ((int64_t)L * N * 12 + (int64_t)e * 12) * 8, 0, 12 * 8 * sizeof(float));
        memset(b->sea_c + ((int64_t)L * N * 12 + (int64_t)e * 12) * 8, 0, 12 * 8 * sizeof(float));
      }
    b->episode_length[e] = 0;
    b->reset[e] = 1;
  }
  int T = nterm_rows(p);
  for (int t = 0; t < T; ++t) {
    float s = 0;
    for (int k = 0; k < n; ++k) s += b->episode_sums[(int64_t)t * N + ids[k]];
    b->extras[t] = (s / (float)n) / p->max_episode_length_s;
    for (int k = 0; k < n; ++k) b->episode_sums[(int64_t)t * N + ids[k]] = 0.0f;
  }
  if (p->curriculum) {
    float s = 0;
    for (int e = 0; e < N; ++e) s += (float)b->terrain_levels[e];
    b->extras[T] = s / (float)N;
  }
  b->extras[T + 1] = (float)n;
  if (p->send_timeouts) memcpy(b->extras_time_outs, b->time_out, (size_t)N);
}

int lgxo_reset_idx(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, const float* draws,
                   const int32_t* ids, int n, int64_t step, int init_done) {
  ctx_t cx = {m, p, b, draws, LGX_DRAW_NOISE + p->num_obs};
  reset_envs(&cx, ids, n, step, 1u, init_done);
  return 0;
}

static void compute_obs(const ctx_t* cx, int e, int64_t step) {
  const lgx_env_params* p = cx->p;
  const lgx_buffers* b = cx->b;
  float* o = b->obs + (int64_t)e * p->num_obs;
  const float* ds = b->dof_state + e * 24;
  const float* c = b->commands + e * 4;
  for (int i = 0; i < 3; ++i) o[i] = b->base_lin_vel[e * 3 + i] * p->obs_scale_lin_vel;
  for (int i = 0; i < 3; ++i) o[3 + i] = b->base_ang_vel[e * 3 + i] * p->obs_scale_ang_vel;
  for (int i = 0; i < 3; ++i) o[6 + i] = b->projected_gravity[e * 3 + i];
  o[9] = c[0] * p->obs_scale_lin_vel; o[10] = c[1] * p->obs_scale_lin_vel; o[11] = c[2] * p->obs_scale_ang_vel;
  for (int j = 0; j < 12; ++j) o[12 + j] = (ds[2 * j] - p->default_dof_pos[j]) * p->obs_scale_dof_pos;
  for (int j = 0; j < 12; ++j) o[24 + j] = ds[2 * j + 1] * p->obs_scale_dof_vel;
  for (int j = 0; j < 12; ++j) o[36 + j] = b->actions[e * 12 + j];
  if (p->measure_heights) {
    float z = b->root_states[e * 13 + 2];
    for (int i = 0; i < p->num_height_points; ++i)
      o[48 + i] = clampf(z - 0.5f - b->measured_heights[e * p->num_height_points + i], -1.0f, 1.0f) * p->obs_scale_height;
  }
  if (p->add_noise)
    for (int i = 0; i < p->num_obs; ++i)
      o[i] += (2.0f * draw(cx, e, LGX_DRAW_NOISE + i, step, 0u) - 1.0f) * p->noise_scale_vec[i];
}

int lgxo_post_physics(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, const float* draws,
                      int64_t step) {
  ctx_t cx = {m, p, b, draws, LGX_DRAW_NOISE + p->num_obs};
  int N = p->num_envs;
  const float gvec[3] = {0.0f, 0.0f, -1.0f};
  const float fwd[3] = {1.0f, 0.0f, 0.0f};
  for (int e = 0; e < N; ++e) {
    b->episode_length[e] += 1;
    float* rs = b->root_states + e * 13;
    quat_rotate_inverse(rs + 3, rs + 7, b->base_lin_vel + e * 3);
    quat_rotate_inverse(rs + 3, rs + 10, b->base_ang_vel + e * 3);
    quat_rotate_inverse(rs + 3, gvec, b->projected_gravity + e * 3);
    /* _post_physics_step_callback :337-352 */
    if (b->episode_length[e] % p->resample_interval == 0) resample_cmd(&cx, e, LGX_DRAW_CMD, step, 0u);
    if (p->heading_command) {
      float f[3]; quat_apply(rs + 3, fwd, f);
      float heading = atan2f(f[1], f[0]);
      b->commands[e * 4 + 2] = clampf(0.5f * wrap_to_pi(b->commands[e * 4 + 3] - heading), -1.0f, 1.0f);
    }
    if (p->measure_heights) get_heights(&cx, e);
  }
  if (p->push_robots && step % p->push_interval == 0)
    for (int e = 0; e < N; ++e)
      for (int i = 0; i < 2; ++i)
        b->root_states[e * 13 + 7 + i] = (p->max_push_vel_xy + p->max_push_vel_xy) * draw(&cx, e, LGX_DRAW_PUSH + i, step, 0u) - p->max_push_vel_xy;
  /* check_termination :143-148 */
  for (int e = 0; e < N; ++e) {
    int r = 0;
    for (int i = 0; i < p->num_termination_bodies; ++i)
      if (norm3(b->contact_forces + (int64_t)e * LGX_MAX_BODIES * 3 + 3 * p->termination_indices[i]) > 1.0f) r = 1;
    b->time_out[e] = (float)b->episode_length[e] > p->max_episode_length;
    b->reset[e] = (uint8_t)(r | b->time_out[e]);
  }
  /* compute_reward :195-212 (per env: its own sums, rew and feet_air_time row) */
#pragma omp parallel for schedule(static)
  for (int e = 0; e < N; ++e) {
    float rew = 0.0f;
    for (int t = 0; t < p->num_terms; ++t) {
      float r = reward_term(&cx, e, p->term_ids[t]) * p->term_scales[t];
      rew += r;
      b->episode_sums[(int64_t)t * N + e] += r;
    }
    if (p->only_positive_rewards && rew < 0.0f) rew = 0.0f;
    if (p->termination_slot >= 0) {
      float r = reward_term(&cx, e, LGX_R_TERMINATION) * p->termination_scale;
      rew += r;
      b->episode_sums[(int64_t)p->termination_slot * N + e] += r;
    }
    b->rew[e] = rew;
  }
  /* reset_idx on reset envs */
  int32_t* ids = (int32_t*)malloc(sizeof(int32_t) * (size_t)N);
  int n = 0;
  for (int e = 0; e < N; ++e) if (b->reset[e]) ids[n++] = e;
  reset_envs(&cx, ids, n, step, 0u, 1);
  free(ids);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < N; ++e) {
    compute_obs(&cx, e, step);
    for (int i = 0; i < p->num_obs; ++i) {
      float* o = b->obs + (int64_t)e * p->num_obs + i;
      *o = clampf(*o, -p->clip_obs, p->clip_obs);
    }
    for (int j = 0; j < 12; ++j) {
      b->last_actions[e * 12 + j] = b->actions[e * 12 + j];
      b->last_dof_vel[e * 12 + j] = b->dof_state[e * 24 + 2 * j + 1];
    }
    for (int i = 0; i < 6; ++i) b->last_root_vel[e * 6 + i] = b->root_states[e * 13 + 7 + i];
  }
  return 0;
}

/* OpenMP threads of the oracle's per-env loops (the CPU baseline states the count it used) */
void lgxo_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

void lgxo_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w);

/* ANYmal's _compute_torques with use_actuator_network (anymal.py:71-78) as the explicit torque
 * source of one substep (LGX_CTRL_SEA): sea_input = [a * action_scale + q0 - q, qd] per joint row
 * (env-major, as sea_input[:, 0, :] = (...).flatten()), one step of the SEA LSTM on the
 * [2, N*12, 8] hidden / cell state, torques clamped to the drive effort limit (PhysX DOF effort
 * mode).  The state of an env that resets is zeroed by reset_envs (anymal.py:56-60). */
static void sea_torques(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, int substep) {
  const int64_t M = (int64_t)p->num_envs * 12;
  float* x = (float*)malloc(sizeof(float) * 2 * M);
  float* tau = (float*)malloc(sizeof(float) * M);
  (void)substep;
  for (int e = 0; e < p->num_envs; ++e) {
    for (int j = 0; j < 12; ++j) {
      const int64_t r = (int64_t)e * 12 + j;
      x[2 * r] = b->actions[r] * p->action_scale + p->default_dof_pos[j] - b->dof_state[2 * r];
      x[2 * r + 1] = b->dof_state[2 * r + 1];
    }
  }
  lgxo_actuator_lstm(x, b->sea_h, b->sea_c, tau, M, b->sea_w);
  for (int64_t r = 0; r < M; ++r) {
    const float eff = m->dof_effort[r % 12];
    b->torques[r] = clampf(tau[r], -eff, eff);
  }
  free(x);
  free(tau);
}

/* the drive inputs of lgxo_step's decimation loop with the dynamics frozen (the golden replay;
 * the HIP lgx_drive_inputs): clip, then per substep the Go1 actuator history (go1.py:79-98) and the
 * position targets (legged_robot.py:394-397), the SEA LSTM torques (anymal.py:71-77, state
 * advanced) or the explicit P / V / T torques (legged_robot.py:370-392), from the unchanged state */
void lgxo_drive_inputs(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b) {
  ctx_t cx = {m, p, b, NULL, 0};
  for (int i = 0; i < p->num_envs * 12; ++i) b->actions[i] = clampf(b->actions[i], -p->clip_actions, p->clip_actions);
  for (int s = 0; s < p->decimation; ++s) {
    cx.substep = s;
    if (p->use_actuator_history)
      for (int e = 0; e < p->num_envs; ++e) actuator_history(&cx, e, s);
    if (p->control_type == LGX_CTRL_POS_DRIVE) lgxo_compute_targets(m, p, b);
    else if (p->control_type == LGX_CTRL_SEA) sea_torques(m, p, b, s);
    else lgxo_explicit_torques(p, b);
  }
}

/* full LeggedRobot.step (legged_robot.py:79-107) */
int lgxo_step(const lgx_model* m, const lgx_env_params* p, const lgx_buffers* b, const float* draws, int64_t step) {
  ctx_t cx = {m, p, b, draws, LGX_DRAW_NOISE + p->num_obs};
  for (int i = 0; i < p->num_envs * 12; ++i) b->actions[i] = clampf(b->actions[i], -p->clip_actions, p->clip_actions);
  for (int s = 0; s < p->decimation; ++s) {
    cx.substep = s;
    if (p->use_actuator_history)
      for (int e = 0; e < p->num_envs; ++e) actuator_history(&cx, e, s);
    if (p->control_type == LGX_CTRL_POS_DRIVE) lgxo_compute_targets(m, p, b);
    else if (p->control_type == LGX_CTRL_SEA) sea_torques(m, p, b, s);
    else lgxo_explicit_torques(p, b);
#pragma omp parallel for schedule(static)
    for (int e = 0; e < p->num_envs; ++e) physics_env(&cx, e);
  }
  return lgxo_post_physics(m, p, b, draws, step);
}

/* ------------------------------------------------------------------ actuator nets */
/* UniNet core MLP on rows of 30 (go1.py:22-35): 30-128-128-128-3 tanh; out *= scale */
void lgxo_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale) {
  const int dims[5] = {30, 128, 128, 128, 3};
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < rows; ++r) {
    float h0[128], h1[128];
    const float* x = in + r * 30;
    float* cur = h0;
    const float* src = x;
    const float* wp = w;
    for (int l = 0; l < 4; ++l) {
      int ni = dims[l], no = dims[l + 1];
      const float* W = wp; const float* B = wp + ni * no; wp = B + no;
      float tmp[128];
      for (int o = 0; o < no; ++o) {
        float s = 0;
        for (int i = 0; i < ni; ++i) s += W[o * ni + i] * src[i];
        s += B[o];
        tmp[o] = l < 3 ? tanhf(s) : s;
      }
      cur = (l & 1) ? h1 : h0;
      memcpy(cur, tmp, no * sizeof(float));
      src = cur;
    }
    for (int o = 0; o < 3; ++o) out[r * 3 + o] = src[o] * out_scale[o];  /* dVel *= vel_std (go1.py:105) */
  }
}

static float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

/* SEA LSTM (anymal.py:62-78; LSTMsea.forward): x*in_scale -> LSTM(2,8,2 layers) -> Linear(8,1) * out_scale.
 * w packed: in_scale[2], out_scale[1], Wih0[32x2], Whh0[32x8], bih0[32], bhh0[32],
 *           Wih1[32x8], Whh1[32x8], bih1[32], bhh1[32], Wlin[8], blin[1] */
void lgxo_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w) {
  const float* in_s = w; const float* out_s = w + 2;
  const float* p = w + 3;
  const float *Wih[2], *Whh[2], *bih[2], *bhh[2];
  Wih[0] = p; p += 64; Whh[0] = p; p += 256; bih[0] = p; p += 32; bhh[0] = p; p += 32;
  Wih[1] = p; p += 256; Whh[1] = p; p += 256; bih[1] = p; p += 32; bhh[1] = p; p += 32;
  const float* Wl = p; const float* bl = p + 8;
  for (int64_t r = 0; r < m; ++r) {
    float inp[8] = {x[r * 2] * in_s[0], x[r * 2 + 1] * in_s[1]};
    int ni = 2;
    for (int L = 0; L < 2; ++L) {
      float* hh = h + ((int64_t)L * m + r) * 8;
      float* cc = c + ((int64_t)L * m + r) * 8;
      float gates[32];
      for (int gi = 0; gi < 32; ++gi) {
        float s = bih[L][gi] + bhh[L][gi];
        for (int i = 0; i < ni; ++i) s += Wih[L][gi * ni + i] * inp[i];
        for (int i = 0; i < 8; ++i) s += Whh[L][gi * 8 + i] * hh[i];
        gates[gi] = s;
      }
      for (int k = 0; k < 8; ++k) {
        float ig = sigm(gates[k]), fg = sigm(gates[8 + k]), gg = tanhf(gates[16 + k]), og = sigm(gates[24 + k]);
        cc[k] = fg * cc[k] + ig * gg;
        hh[k] = og * tanhf(cc[k]);
      }
      memcpy(inp, hh, 8 * sizeof(float));
      ni = 8;
    }
    float s = bl[0];
    for (int i = 0; i < 8; ++i) s += Wl[i] * inp[i];
    tau[r] = out_s[0] * s;
  }
}
#endif /* LGXO_PHYSICS_ONLY */
