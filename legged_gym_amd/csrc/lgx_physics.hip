// lgx physics kernel: `decimation` fused substeps of floating-base 4x3-DoF articulated
// dynamics with implicit PD drives, joint-limit springs and compliant ground contact.
// Replaces Isaac Gym PhysX `gym.simulate` as driven by LeggedRobot.step
// (legged_robot.py:89-99; model/drive setup legged_robot.py:645-740).  Model: DESIGN.md §3.
//
// Mapping (CDNA4, wave64), lgx_physics_kernel<PP>: one env per 4 PP lanes, lane = leg x PP-way
// split of the leg's contact candidates (PP = 4 at every size: 16 lanes per env, 4 envs per wave,
// 16 envs per 256-thread workgroup).  The joint-space mass matrix of a quadruped is "arrowhead": a
// 6x6 base block A coupled to four independent 3x3 leg blocks D_l through 6x3 blocks B_l.  Each lane
// builds its leg's B_l/D_l (composite-rigid-body algorithm on a 3-link chain), its leg's bias forces
// (RNEA) and its share of the leg's contact terms (reduced over the PP lanes with DPP row sums); the
// base Schur complement A - sum_l B_l D_l^-1 B_l^T is formed with quad shuffles and its 6x6 Cholesky
// solved redundantly by every lane of the env; the leg back-substitution is lane-local again.
// Per-substep state stays in VGPRs, leg-uniform values and the heightfield patch in LDS; HBM
// traffic per env-step = state in + state out (+ actuator-net history).
// lgx_physics_dense_kernel (end of file): the biped's 2 x 6 chains (and any robot with
// LGX_PHYS_DENSE=1), one env per wavefront, the oracle's dense algorithm.
#include <stdlib.h>

#include "lgx_device.h"
#include "lgx_internal.h"

namespace {

struct sv { f3 a, l; };  // spatial vector (angular; linear), reference point = base origin O
LGX_DEV sv sv0() { return sv{mk3(0, 0, 0), mk3(0, 0, 0)}; }
LGX_DEV sv add(sv x, sv y) { return sv{x.a + y.a, x.l + y.l}; }
LGX_DEV sv scale(float s, sv x) { return sv{s * x.a, s * x.l}; }
LGX_DEV float dot(sv x, sv y) { return dot(x.a, y.a) + dot(x.l, y.l); }
LGX_DEV sv crm(sv V, sv s) { return sv{cross(V.a, s.a), cross(V.a, s.l) + cross(V.l, s.a)}; }
LGX_DEV sv crf(sv V, sv f) { return sv{cross(V.a, f.a) + cross(V.l, f.l), cross(V.a, f.l)}; }

// compact spatial inertia about O: [[Ibar, skew(h)], [skew(h)^T, m 1]], h = m c
struct SI { float m; f3 h; float I[6]; };  // I: xx yy zz xy xz yz
LGX_DEV SI si_add(const SI& x, const SI& y) {
  SI r; r.m = x.m + y.m; r.h = x.h + y.h;
#pragma unroll
  for (int i = 0; i < 6; ++i) r.I[i] = x.I[i] + y.I[i];
  return r;
}
LGX_DEV sv si_mul(const SI& s, sv v) {
  f3 Ia = mk3(s.I[0] * v.a.x + s.I[3] * v.a.y + s.I[4] * v.a.z, s.I[3] * v.a.x + s.I[1] * v.a.y + s.I[5] * v.a.z,
              s.I[4] * v.a.x + s.I[5] * v.a.y + s.I[2] * v.a.z);
  return sv{Ia + cross(s.h, v.l), cross(v.a, s.h) + s.m * v.l};
}
LGX_DEV SI body_si(const lgx_model* __restrict__ M, int b, float scale, const m33& R, f3 o) {
  const float* in = M->body_inertia[b];
  m33 Ib = {{in[0], in[3], in[4], in[3], in[1], in[5], in[4], in[5], in[2]}};
  m33 T = mul(R, Ib);
  float Iw[6];  // T R^T, symmetric part
  Iw[0] = T.a[0] * R.a[0] + T.a[1] * R.a[1] + T.a[2] * R.a[2];
  Iw[1] = T.a[3] * R.a[3] + T.a[4] * R.a[4] + T.a[5] * R.a[5];
  Iw[2] = T.a[6] * R.a[6] + T.a[7] * R.a[7] + T.a[8] * R.a[8];
  Iw[3] = T.a[0] * R.a[3] + T.a[1] * R.a[4] + T.a[2] * R.a[5];
  Iw[4] = T.a[0] * R.a[6] + T.a[1] * R.a[7] + T.a[2] * R.a[8];
  Iw[5] = T.a[3] * R.a[6] + T.a[4] * R.a[7] + T.a[5] * R.a[8];
  f3 c = o + mul(R, mk3(M->body_com[b][0], M->body_com[b][1], M->body_com[b][2]));
  float m = M->body_mass[b] * scale;
  float cc = dot(c, c);
  SI s;
  s.m = m;
  s.h = m * c;
  s.I[0] = Iw[0] * scale + m * (cc - c.x * c.x);
  s.I[1] = Iw[1] * scale + m * (cc - c.y * c.y);
  s.I[2] = Iw[2] * scale + m * (cc - c.z * c.z);
  s.I[3] = Iw[3] * scale - m * c.x * c.y;
  s.I[4] = Iw[4] * scale - m * c.x * c.z;
  s.I[5] = Iw[5] * scale - m * c.y * c.z;
  return s;
}

// packed symmetric 6x6 (upper triangle, row-major): idx(i,j), i<=j
LGX_DEV constexpr int sidx(int i, int j) { return i <= j ? (i * 11 - i * i) / 2 + j : (j * 11 - j * j) / 2 + i; }

LGX_DEV void si_to_sym6(const SI& s, float* A) {  // A[21]
  A[sidx(0, 0)] = s.I[0]; A[sidx(1, 1)] = s.I[1]; A[sidx(2, 2)] = s.I[2];
  A[sidx(0, 1)] = s.I[3]; A[sidx(0, 2)] = s.I[4]; A[sidx(1, 2)] = s.I[5];
  // top-right skew(h): [[0,-hz,hy],[hz,0,-hx],[-hy,hx,0]]
  A[sidx(0, 3)] = 0.f;     A[sidx(0, 4)] = -s.h.z; A[sidx(0, 5)] = s.h.y;
  A[sidx(1, 3)] = s.h.z;   A[sidx(1, 4)] = 0.f;    A[sidx(1, 5)] = -s.h.x;
  A[sidx(2, 3)] = -s.h.y;  A[sidx(2, 4)] = s.h.x;  A[sidx(2, 5)] = 0.f;
  A[sidx(3, 3)] = s.m; A[sidx(4, 4)] = s.m; A[sidx(5, 5)] = s.m;
  A[sidx(3, 4)] = 0.f; A[sidx(3, 5)] = 0.f; A[sidx(4, 5)] = 0.f;
}

LGX_DEV float sv_get(const sv& v, int i) {
  return i == 0 ? v.a.x : i == 1 ? v.a.y : i == 2 ? v.a.z : i == 3 ? v.l.x : i == 4 ? v.l.y : v.l.z;
}

// Transcendentals on the per-substep critical path (the 6x6 Cholesky's pivots, the leg blocks'
// inverse determinant, the joint rotations): the hardware v_rsq_f32 / v_rcp_f32 / v_sin_f32 /
// v_cos_f32 (~1 ulp; 1 instruction each) instead of the correctly rounded sequences (~8-40
// dependent instructions each: a chain of 8 arrow solves x 6 pivots per launch at one wave per
// SIMD).  -DLGX_PHYS_FAST_TRANSC=0 restores the correctly rounded forms (A/B; the oracle uses them).
#ifndef LGX_PHYS_FAST_TRANSC
#define LGX_PHYS_FAST_TRANSC 1
#endif

// 6x6 SPD solve (packed sym), in registers
// (the substitutions multiply by the factorisation's reciprocal diagonal: 12 of the 18 correctly
// rounded divisions of the textbook form, ~10 instructions each, on the per-substep critical path)
LGX_DEV void chol6_solve(float* A, float* b) {
  float L[21], Li[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float s = A[sidx(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[sidx(j, k)] * L[sidx(j, k)];
#if LGX_PHYS_FAST_TRANSC
    const float sc = fmaxf(s, 1e-20f);
    const float inv = __builtin_amdgcn_rsqf(sc);   // pivot 1 / sqrt(s) and sqrt(s) = s / sqrt(s)
    const float d = sc * inv;
#else
    float d = sqrtf(fmaxf(s, 1e-20f));
    const float inv = 1.0f / d;
#endif
    L[sidx(j, j)] = d;
    Li[j] = inv;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      float t = A[sidx(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[sidx(i, k)] * L[sidx(j, k)];
      L[sidx(i, j)] = t * inv;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[sidx(i, k)] * b[k];
    b[i] = t * Li[i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    float t = b[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) t -= L[sidx(k, i)] * b[k];
    b[i] = t * Li[i];
  }
}

// Rodrigues rotation with the hardware sine / cosine (v_sin_f32 / v_cos_f32 on th / 2 pi)
LGX_DEV m33 axis_angle_hw(f3 a, float th) {
  const float s = __sinf(th), c = __cosf(th);
  const float t = 1 - c;
  m33 R;
  R.a[0] = t * a.x * a.x + c;       R.a[1] = t * a.x * a.y - s * a.z; R.a[2] = t * a.x * a.z + s * a.y;
  R.a[3] = t * a.x * a.y + s * a.z; R.a[4] = t * a.y * a.y + c;       R.a[5] = t * a.y * a.z - s * a.x;
  R.a[6] = t * a.x * a.z - s * a.y; R.a[7] = t * a.y * a.z + s * a.x; R.a[8] = t * a.z * a.z + c;
  return R;
}

// reciprocal / reciprocal square root / quotient of the contact queries (per candidate and substep):
// v_rcp_f32 / v_rsq_f32 (~1 ulp) under LGX_PHYS_FAST_TRANSC, the correctly rounded forms otherwise
LGX_DEV float ph_rcp(float x) {
#if LGX_PHYS_FAST_TRANSC
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
LGX_DEV float ph_rsqrt(float x) {
#if LGX_PHYS_FAST_TRANSC
  return __builtin_amdgcn_rsqf(x);
#else
  return 1.0f / sqrtf(x);
#endif
}
LGX_DEV float ph_div(float a, float b) {
#if LGX_PHYS_FAST_TRANSC
  return a * __builtin_amdgcn_rcpf(b);
#else
  return a / b;
#endif
}

// inverse of a symmetric positive-definite 3x3 (packed d00 d11 d22 d01 d02 d12)
LGX_DEV void inv3sym(const float* D, float* Di) {
  float c00 = D[1] * D[2] - D[5] * D[5];
  float c01 = D[4] * D[5] - D[3] * D[2];
  float c02 = D[3] * D[5] - D[4] * D[1];
  float det = D[0] * c00 + D[3] * c01 + D[4] * c02;
#if LGX_PHYS_FAST_TRANSC
  float id = __builtin_amdgcn_rcpf(det);
#else
  float id = 1.0f / det;
#endif
  Di[0] = c00 * id;
  Di[3] = c01 * id;
  Di[4] = c02 * id;
  Di[1] = (D[0] * D[2] - D[4] * D[4]) * id;
  Di[5] = (D[3] * D[4] - D[0] * D[5]) * id;
  Di[2] = (D[0] * D[1] - D[3] * D[3]) * id;
}
LGX_DEV f3 sym3_mul(const float* D, f3 x) {
  return mk3(D[0] * x.x + D[3] * x.y + D[4] * x.z, D[3] * x.x + D[1] * x.y + D[5] * x.z,
             D[4] * x.x + D[5] * x.y + D[2] * x.z);
}

// Jacobian column c (0..5) of the base part of a point velocity v_P = v + w x P: e_c x P | e_{c-3}
LGX_DEV f3 jb_col(int c, f3 P) {
  return c == 0 ? mk3(0.f, -P.z, P.y) : c == 1 ? mk3(P.z, 0.f, -P.x) : c == 2 ? mk3(-P.y, P.x, 0.f)
       : c == 3 ? mk3(1.f, 0.f, 0.f) : c == 4 ? mk3(0.f, 1.f, 0.f) : mk3(0.f, 0.f, 1.f);
}

LGX_DEV m33 sel3(int k, const m33& a, const m33& b, const m33& c) {
  m33 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.a[i] = k == 0 ? a.a[i] : (k == 1 ? b.a[i] : c.a[i]);
  return r;
}
LGX_DEV f3 sel3(int k, f3 a, f3 b, f3 c) { return k == 0 ? a : (k == 1 ? b : c); }
LGX_DEV sv sel3(int k, const sv& a, const sv& b, const sv& c) { return sv{sel3(k, a.a, b.a, c.a), sel3(k, a.l, b.l, c.l)}; }

struct LegSys {     // lane-private pieces of the arrowhead system
  float Ap[21];     // base-block additions from this lane (contacts)
  float B[6][3];    // base-leg coupling
  float D[6];       // leg block (packed sym 3x3)
  float rb[6];      // base rhs partial
  float rl[3];      // leg rhs
};

// adds J^T W J and J^T f for a point P on leg body `k` (k = -1: base), W = wt*I + (wn - wt) n n^T.
// Column j of W J is formed on the fly (3 floats live instead of 27).
LGX_DEV void add_contact(LegSys& L, f3 P, f3 n, float wn, float wt, f3 f, int k, const sv* S) {
  f3 Jc[9];  // 6 base + up to 3 leg columns
#pragma unroll
  for (int c = 0; c < 6; ++c) Jc[c] = jb_col(c, P);
#pragma unroll
  for (int j = 0; j < 3; ++j) Jc[6 + j] = (j <= k) ? cross(S[j].a, P) + S[j].l : mk3(0.f, 0.f, 0.f);
  const float dw = wn - wt;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const f3 wj = wt * Jc[j] + (dw * dot(n, Jc[j])) * n;
    if (j < 6) {
#pragma unroll
      for (int i = 0; i <= j; ++i) L.Ap[sidx(i, j)] += dot(Jc[i], wj);
    } else {
      const int jl = j - 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) L.B[i][jl] += dot(Jc[i], wj);
      if (jl == 0) L.D[0] += dot(Jc[6], wj);
      if (jl == 1) { L.D[1] += dot(Jc[7], wj); L.D[3] += dot(Jc[6], wj); }
      if (jl == 2) { L.D[2] += dot(Jc[8], wj); L.D[4] += dot(Jc[6], wj); L.D[5] += dot(Jc[7], wj); }
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) L.rb[i] += dot(Jc[i], f);
#pragma unroll
  for (int j = 0; j < 3; ++j) L.rl[j] += dot(Jc[6 + j], f);
}

// solve the arrowhead system; returns base solution xb[6] (all lanes) and leg solution xl
LGX_DEV void arrow_solve(LegSys& L, const float* Acommon, const float* rbcommon, bool lane0, float* xb, f3& xl) {
  float Di[6];
  inv3sym(L.D, Di);
  // Y = Di B^T (3x6); Schur partial = Ap - B Y ; rb partial = rb - B Di rl
  f3 Y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) Y[i] = sym3_mul(Di, mk3(L.B[i][0], L.B[i][1], L.B[i][2]));
  f3 Dr = sym3_mul(Di, mk3(L.rl[0], L.rl[1], L.rl[2]));
  // the env's common base block enters on the leg-0 lane: every lane reads it (one broadcast LDS
  // address) and selects the sum - a read under `if (lane0)` compiles to a branch with its own
  // lgkmcnt(0) wait, 27 serial LDS round trips per solve
  float A[21], rb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = i; j < 6; ++j) {
      const float ac = Acommon[sidx(i, j)];
      const float v = L.Ap[sidx(i, j)] - (L.B[i][0] * Y[j].x + L.B[i][1] * Y[j].y + L.B[i][2] * Y[j].z);
      A[sidx(i, j)] = quad_sum(lane0 ? v + ac : v);
    }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float rc = rbcommon[i];
    const float v = L.rb[i] - (L.B[i][0] * Dr.x + L.B[i][1] * Dr.y + L.B[i][2] * Dr.z);
    rb[i] = quad_sum(lane0 ? v + rc : v);
  }
  chol6_solve(A, rb);
#pragma unroll
  for (int i = 0; i < 6; ++i) xb[i] = rb[i];
  f3 t = mk3(L.rl[0], L.rl[1], L.rl[2]);
#pragma unroll
  for (int i = 0; i < 6; ++i) t = t - xb[i] * mk3(L.B[i][0], L.B[i][1], L.B[i][2]);
  xl = sym3_mul(Di, t);
}

// One step of the ANYmal SEA actuator network for joint row r of m (anymal.py:71-78; upstream
// LSTMsea.forward): x = [a*s + q0 - q, qd] * in_scale -> 2-layer LSTM(2 -> 8) -> Linear(8 -> 1) *
// out_scale; torch gate order i, f, g, o.  Hidden / cell state in place in global memory ([2, m, 8]:
// the reference's sea_hidden_state layout, L2-resident across the substeps; zeroed for envs that
// reset by the post-physics reset_env, anymal.py:56-60); `store`: write the new state (false for
// padding lanes).  Weights are uniform
// (scalar loads).  Sigmoid 1/(1+exp(-x)) and tanh 1 - 2/(exp(2x)+1) on v_exp_f32 (|err| <= ~2e-7).
LGX_DEV float sea_sigm(float x) { return 1.f / (1.f + __expf(-x)); }
LGX_DEV float sea_tanh(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }
LGX_DEV float sea_lstm(const float* __restrict__ w, float* __restrict__ h, float* __restrict__ c, int64_t r,
                       int64_t m, float x0, float x1, bool store) {
  const float* Wl = w + 3 + 64 + 256 + 32 + 32 + 256 + 256 + 32 + 32;
  float inp[8] = {x0 * w[0], x1 * w[1], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int L = 0; L < 2; ++L) {
    const int ni = L ? 8 : 2;
    const float* Wih = w + 3 + (L ? 64 + 256 + 64 : 0);
    const float* Whh = Wih + 32 * ni;
    const float* bih = Whh + 256;
    const float* bhh = bih + 32;
    float4* hp = reinterpret_cast<float4*>(h + ((int64_t)L * m + r) * 8);
    float4* cp = reinterpret_cast<float4*>(c + ((int64_t)L * m + r) * 8);
    float4 h0 = hp[0], h1 = hp[1], c0 = cp[0], c1 = cp[1];
    const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    float g[32];
#pragma unroll
    for (int gi = 0; gi < 32; ++gi) {
      float sg = bih[gi] + bhh[gi];
#pragma unroll
      for (int i = 0; i < ni; ++i) sg += Wih[gi * ni + i] * inp[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) sg += Whh[gi * 8 + i] * hv[i];
      g[gi] = sg;
    }
    float hn[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cv[k] = sea_sigm(g[8 + k]) * cv[k] + sea_sigm(g[k]) * sea_tanh(g[16 + k]);
      hn[k] = sea_sigm(g[24 + k]) * sea_tanh(cv[k]);
      inp[k] = hn[k];
    }
    if (store) {
      hp[0] = make_float4(hn[0], hn[1], hn[2], hn[3]);
      hp[1] = make_float4(hn[4], hn[5], hn[6], hn[7]);
      cp[0] = make_float4(cv[0], cv[1], cv[2], cv[3]);
      cp[1] = make_float4(cv[4], cv[5], cv[6], cv[7]);
    }
  }
  float t = Wl[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t += Wl[i] * inp[i];
  return w[2] * t;
}

// ---- contact against the slope-corrected trimesh (terrain.py:70-73; the mesh of legged_robot.py:629-643)
// closest point of triangle abc to p (Voronoi-region walk: Ericson, Real-Time Collision Detection 5.1.5)
LGX_DEV f3 closest_on_tri(f3 p, f3 a, f3 b, f3 c) {
  const f3 ab = b - a, ac = c - a, ap = p - a;
  const float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) return a;
  const f3 bp = p - b;
  const float d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.f && d4 <= d3) return b;
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) return a + ph_div(d1, d1 - d3) * ab;
  const f3 cq = p - c;
  const float d5 = dot(ab, cq), d6 = dot(ac, cq);
  if (d6 >= 0.f && d5 <= d6) return c;
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) return a + ph_div(d2, d2 - d6) * ac;
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) return b + ph_div(d4 - d3, (d4 - d3) + (d5 - d6)) * (c - b);
  const float den = ph_rcp(va + vb + vc);
  return a + (vb * den) * ab + (vc * den) * ac;
}

// one triangle of the query: nearest point so far (squared distance, point, the face's cross
// product) and the highest surface among the triangles whose xy projection holds p (height, cross
// product); face normals are normalised only for the rare on-surface case at the end
struct TmQuery { float d2; f3 cp, cn; float top; f3 tn; };
LGX_DEV void tm_tri(TmQuery& q, f3 p, f3 a, f3 b, f3 c) {
  const f3 cp = closest_on_tri(p, a, b, c);
  const f3 dv = p - cp;
  const float d2 = dot(dv, dv);
  const f3 e1 = b - a, e2 = c - a;
  if (d2 < q.d2) { q.d2 = d2; q.cp = cp; q.cn = cross(e1, e2); }
  const float den = e1.x * e2.y - e1.y * e2.x;      // 2 x signed xy area (0 for vertical faces)
  if (fabsf(den) > 1e-9f) {
    const float id = ph_rcp(den);
    const float px = p.x - a.x, py = p.y - a.y;
    const float s = (px * e2.y - py * e2.x) * id, t = (e1.x * py - e1.y * px) * id;
    if (s >= -1e-6f && t >= -1e-6f && s + t <= 1.f + 1e-6f) {
      const float hz = a.z + s * e1.z + t * e2.z;
      if (hz > q.top) { q.top = hz; q.tn = cross(e1, e2); }
    }
  }
}

// the 4 x 4 vertex block around cell (i, j) (rows i-1 .. i+2, cols j-1 .. j+2; clamped at the map
// edge): heights and move codes.  One branch around each source's 16 loads (a per-load condition
// compiles to a branch and a full wait after every load: 16 serial round trips)
LGX_DEV void tm_block(const lgx_buffers& B, int i, int j, const int32_t* hpatch, int pi0, int pj0, int* hv, int* cd) {
  const int rows = B.hf_rows, cols = B.hf_cols;
  const bool in_patch = hpatch && (unsigned)(i - 1 - pi0) < LGX_HF_PATCH - 3 && (unsigned)(j - 1 - pj0) < LGX_HF_PATCH - 3;
  if (in_patch) {
    const int32_t* q = hpatch + (i - 1 - pi0) * LGX_HF_PATCH + (j - 1 - pj0);
    int w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = q[(k >> 2) * LGX_HF_PATCH + (k & 3)];
#pragma unroll
    for (int k = 0; k < 16; ++k) { hv[k] = w[k] >> 8; cd[k] = w[k] & 15; }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int a = min(max(i - 1 + (k >> 2), 0), rows - 1), b = min(max(j - 1 + (k & 3), 0), cols - 1);
      hv[k] = B.height_samples[(int64_t)a * cols + b];
      cd[k] = B.hf_trimesh[(int64_t)a * cols + b];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) cd[k] &= 15;
  }
}

// the cell (i, j) under world point p (clamped to the map)
LGX_DEV void tm_cell(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, int* i, int* j) {
  const float ihs = 1.0f / P->horizontal_scale;
  const float u = (p.x + P->border_size) * ihs, v = (p.y + P->border_size) * ihs;
  *i = min(max((int)floorf(u), 0), B.hf_rows - 2);
  *j = min(max((int)floorf(v), 0), B.hf_cols - 2);
}

// The corrected-mesh query is built from three pieces shared by the one-lane form (trimesh_depth) and
// the 16-lanes-per-query form of the physics kernel, so both round identically:
// tm_local: the geometry in a frame at raw vertex (i, j) (coordinates of a few cells: float precision
// of the nearest point and normal independent of how far the env is from the world origin); no fma
// contraction in the frame change, so the oracle's restatement rounds identically
LGX_DEV f3 tm_local(const lgx_env_params* __restrict__ P, f3 p, int i, int j) {
  const float hs = P->horizontal_scale, bo = P->border_size;
  const float ox = __fsub_rn(__fmul_rn((float)i, hs), bo), oy = __fsub_rn(__fmul_rn((float)j, hs), bo);
  return mk3(__fsub_rn(p.x, ox), __fsub_rn(p.y, oy), p.z);
}

// tm_cell_tris: cell (ca, cb) of the 3 x 3 around (i, j) (ca, cb in 0..2) against local point p: its 4
// samples (LDS patch or global), moved vertices, cull (off the map; p more than r above every vertex
// of the cell - no contact, not below its surface; or outside its xy box grown by r - farther than r,
// not over it), then its two triangles into q in the reference order
LGX_DEV void tm_cell_tris(TmQuery& q, const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, int i,
                          int j, int ca, int cb, const int32_t* hpatch, int pi0, int pj0) {
  const float hs = P->horizontal_scale, vs = P->vertical_scale;
  const int rows = B.hf_rows, cols = B.hf_cols;
  const int ci = i - 1 + ca, cj = j - 1 + cb;
  if (ci < 0 || ci > rows - 2 || cj < 0 || cj > cols - 2) return;
  int h[4], code[4];   // samples (ci + (k & 1), cj + (k >> 1))
  if (hpatch && (unsigned)(ci - pi0) < LGX_HF_PATCH - 1 && (unsigned)(cj - pj0) < LGX_HF_PATCH - 1) {
    const int32_t* w = hpatch + (ci - pi0) * LGX_HF_PATCH + (cj - pj0);
    const int w0 = w[0], w1 = w[LGX_HF_PATCH], w2 = w[1], w3 = w[LGX_HF_PATCH + 1];
    h[0] = w0 >> 8; h[1] = w1 >> 8; h[2] = w2 >> 8; h[3] = w3 >> 8;
    code[0] = w0 & 15; code[1] = w1 & 15; code[2] = w2 & 15; code[3] = w3 & 15;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t o = (int64_t)(ci + (k & 1)) * cols + cj + (k >> 1);
      h[k] = B.height_samples[o];
      code[k] = B.hf_trimesh[o];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) code[k] &= 15;
  }
  f3 v[4];   // (ci, cj), (ci + 1, cj), (ci, cj + 1), (ci + 1, cj + 1)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int da = ca + (k & 1), db = cb + (k >> 1);
    const int dx = ((code[k] * 11) >> 5) - 1, dy = code[k] - 3 * (dx + 1) - 1;
    v[k] = mk3((float)(da - 1 + dx) * hs, (float)(db - 1 + dy) * hs, (float)h[k] * vs);
  }
  const float zmax = fmaxf(fmaxf(v[0].z, v[1].z), fmaxf(v[2].z, v[3].z));
  const float xmin = fminf(fminf(v[0].x, v[1].x), fminf(v[2].x, v[3].x)), xmax = fmaxf(fmaxf(v[0].x, v[1].x), fmaxf(v[2].x, v[3].x));
  const float ymin = fminf(fminf(v[0].y, v[1].y), fminf(v[2].y, v[3].y)), ymax = fmaxf(fmaxf(v[0].y, v[1].y), fmaxf(v[2].y, v[3].y));
  if (p.z - r > zmax || p.x < xmin - r || p.x > xmax + r || p.y < ymin - r || p.y > ymax + r) return;
  tm_tri(q, p, v[0], v[3], v[2]);   // reference triangle order (ind0, ind3, ind1), (ind0, ind2, ind3)
  tm_tri(q, p, v[0], v[1], v[3]);
}

LGX_DEV void tm_init(TmQuery& q, f3 p) {
  q.d2 = 3.0e38f; q.cp = p; q.cn = mk3(0.f, 0.f, 1.f);
  q.top = -3.0e38f; q.tn = mk3(0.f, 0.f, 1.f);
}

// tm_finish: inside = p below the surface under it; depth = r -/+ distance, normal = from the surface
// point toward p (outside) or from p toward it (inside); where p sits on the surface, the face normal
LGX_DEV float tm_finish(const TmQuery& q, f3 p, float r, f3* n) {
  const bool inside = p.z < q.top;
  const float d = sqrtf(q.d2);
  if (d > 1e-7f) {
    const float inv = ph_rcp(d);
    *n = inside ? inv * (q.cp - p) : inv * (p - q.cp);
  } else {
    f3 c = q.top > -1e30f ? q.tn : q.cn;
    c = (c.z < 0.f ? -1.f : 1.f) / fmaxf(sqrtf(dot(c, c)), 1e-30f) * c;   // face normal, oriented up
    *n = c;
  }
  return inside ? r + d : r - d;
}

// false when the sphere is more than r above every vertex of the 4 x 4 block around its cell (i, j)
// (no face within r, not below the surface): the query's early out on its own
LGX_DEV bool tm_near(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, int i, int j,
                     const int32_t* hpatch, int pi0, int pj0) {
  int hv[16], cd[16];
  tm_block(B, i, j, hpatch, pi0, pj0, hv, cd);
  int hmax = hv[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) hmax = max(hmax, hv[k]);
  return !(p.z - r > (float)hmax * P->vertical_scale);
}

// tm_keep: the cells of the 3 x 3 around p's cell (i, j) the query has to visit (bit ca * 3 + cb):
// 0 when p is more than r above every vertex of the 4 x 4 block (the spheres off the ground) or every
// cell is culled (tm_cell_tris' tests, here on the block decoded once in registers) - no face within
// r and p not below the surface: no contact.  `pl` returns p in the local frame.
LGX_DEV unsigned tm_keep(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, int i, int j,
                         const int32_t* hpatch, int pi0, int pj0, f3* pl) {
  const float hs = P->horizontal_scale, vs = P->vertical_scale;
  const int rows = B.hf_rows, cols = B.hf_cols;
  int hv[16], cd[16];
  tm_block(B, i, j, hpatch, pi0, pj0, hv, cd);
  int hmax = hv[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) hmax = max(hmax, hv[k]);
  p = tm_local(P, p, i, j);
  *pl = p;
  if (p.z - r > (float)hmax * vs) return 0u;
  unsigned keep = 0;
#pragma unroll
  for (int ca = 0; ca < 3; ++ca)
#pragma unroll
    for (int cb = 0; cb < 3; ++cb) {
      const int ci = i - 1 + ca, cj = j - 1 + cb;
      f3 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int da = ca + (k & 1), db = cb + (k >> 1);
        const int code = cd[da * 4 + db];
        const int dx = ((code * 11) >> 5) - 1, dy = code - 3 * (dx + 1) - 1;
        v[k] = mk3((float)(da - 1 + dx) * hs, (float)(db - 1 + dy) * hs, (float)hv[da * 4 + db] * vs);
      }
      const float zmax = fmaxf(fmaxf(v[0].z, v[1].z), fmaxf(v[2].z, v[3].z));
      const float xmin = fminf(fminf(v[0].x, v[1].x), fminf(v[2].x, v[3].x)), xmax = fmaxf(fmaxf(v[0].x, v[1].x), fmaxf(v[2].x, v[3].x));
      const float ymin = fminf(fminf(v[0].y, v[1].y), fminf(v[2].y, v[3].y)), ymax = fmaxf(fmaxf(v[0].y, v[1].y), fmaxf(v[2].y, v[3].y));
      const bool on_map = ci >= 0 && ci <= rows - 2 && cj >= 0 && cj <= cols - 2;
      const bool cull = p.z - r > zmax || p.x < xmin - r || p.x > xmax + r || p.y < ymin - r || p.y > ymax + r;
      if (on_map && !cull) keep |= 1u << (ca * 3 + cb);
    }
  return keep;
}

// the kept cells of a query in cell order (the sequential scan: strict comparisons, first triangle kept)
LGX_DEV float tm_visit(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 pl, float r, int i, int j,
                       unsigned keep, f3* n, const int32_t* hpatch, int pi0, int pj0) {
  TmQuery q;
  tm_init(q, pl);
  while (keep) {
    const int c = __builtin_ctz(keep);
    keep &= keep - 1;
    const int ca = (c * 11) >> 5;   // c / 3 for c < 9
    tm_cell_tris(q, P, B, pl, r, i, j, ca, c - 3 * ca, hpatch, pi0, pj0);
  }
  return tm_finish(q, pl, r, n);
}

// Signed contact depth of a sphere (radius r >= 0, centre p, world frame) against the corrected
// mesh around cell (i, j): the nearest surface point over the two triangles of each cell of the
// 3 x 3 cells around (i, j) (the moves are at most one cell, so every face within r < one cell of
// p is among them) that the culls keep, in cell order; -1 (normal up) when no cell is kept.
LGX_DEV float trimesh_depth(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, int i, int j,
                            f3* n, const int32_t* hpatch, int pi0, int pj0) {
  f3 pl;
  const unsigned keep = tm_keep(P, B, p, r, i, j, hpatch, pi0, pj0, &pl);
  if (!keep) { *n = mk3(0.f, 0.f, 1.f); return -1.f; }
  return tm_visit(P, B, pl, r, i, j, keep, n, hpatch, pi0, pj0);
}

// the query state of the lane 16 - `m` lanes away in a 16-lane row (xor m, DPP), as floats
template <int M>
LGX_DEV float row_xor(float v) {
  return M == 1 ? lane_xor1(v) : M == 2 ? lane_xor2(v) : M == 4 ? lane_xor4(v) : lane_xor8(v);
}
// combine the per-cell query states of a 16-lane row (lane g holds cell g, g < 9): the smallest
// distance and the highest covering surface, ties to the lower cell - the order of the sequential
// scan (strict comparisons, first triangle kept), so the result equals trimesh_depth's
template <int M>
LGX_DEV void tm_combine_step(TmQuery& q, int& cd2, int& ctop) {
  const float od2 = row_xor<M>(q.d2), otop = row_xor<M>(q.top);
  const int ocd2 = __builtin_bit_cast(int, row_xor<M>(__builtin_bit_cast(float, cd2)));
  const int octop = __builtin_bit_cast(int, row_xor<M>(__builtin_bit_cast(float, ctop)));
  const f3 ocp = mk3(row_xor<M>(q.cp.x), row_xor<M>(q.cp.y), row_xor<M>(q.cp.z));
  const f3 ocn = mk3(row_xor<M>(q.cn.x), row_xor<M>(q.cn.y), row_xor<M>(q.cn.z));
  const f3 otn = mk3(row_xor<M>(q.tn.x), row_xor<M>(q.tn.y), row_xor<M>(q.tn.z));
  if (od2 < q.d2 || (od2 == q.d2 && ocd2 < cd2)) { q.d2 = od2; q.cp = ocp; q.cn = ocn; cd2 = ocd2; }
  if (otop > q.top || (otop == q.top && octop < ctop)) { q.top = otop; q.tn = otn; ctop = octop; }
}

// Ground contact of a sphere / point (radius r) centred at world p, first stage: spheres (r > 0: feet,
// capsule ends) on a cell its contact table flags (near a moved vertex) need the corrected-trimesh
// query (`*defer` = true, depth not computed); everything else is answered here against the
// triangulated heightfield under p (identical where no vertex of the neighbourhood moved), depth
// along its face normal.  Box corners (r = 0) keep the heightfield query everywhere: on a fallen
// robot dozens of them sit near the ground, and the full query per point (up to 18 triangles,
// latency-bound at one wave per SIMD) cost 2x the whole physics launch.
LGX_DEV float ground_cell(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, f3* n,
                          const int32_t* patch, int pi0, int pj0, bool* defer) {
  *defer = false;
  if (P->terrain_kind == 0 || B.height_samples == nullptr) { *n = mk3(0.f, 0.f, 1.f); return r - p.z; }
  // cell and slopes on the reciprocal of the horizontal scale (uniform: one division per launch, not
  // four correctly rounded ones per query; the oracle rounds the same way)
  const float ihs = 1.0f / P->horizontal_scale, vs = P->vertical_scale;
  const float u = (p.x + P->border_size) * ihs, v = (p.y + P->border_size) * ihs;
  const int i = min(max((int)floorf(u), 0), B.hf_rows - 2), j = min(max((int)floorf(v), 0), B.hf_cols - 2);
  // the cell's 4 samples (height << 8 | contact-table byte in the LDS patch) in one round trip
  int q00, q10, q01, q11;
  const int li = i - pi0, lj = j - pj0;
  if (patch && (unsigned)li < LGX_HF_PATCH - 1 && (unsigned)lj < LGX_HF_PATCH - 1) {
    const int32_t* q = patch + li * LGX_HF_PATCH + lj;
    q00 = q[0]; q10 = q[LGX_HF_PATCH]; q01 = q[1]; q11 = q[LGX_HF_PATCH + 1];
  } else {
    const int16_t* H = B.height_samples;
    const int64_t o = (int64_t)i * B.hf_cols + j;
    const int tb = B.hf_trimesh ? B.hf_trimesh[o] & 0xff : 4;
    q00 = (H[o] << 8) | tb; q10 = H[o + B.hf_cols] << 8; q01 = H[o + 1] << 8; q11 = H[o + B.hf_cols + 1] << 8;
  }
  if (r > 0.f && B.hf_trimesh && (q00 & 16)) { *defer = true; return 0.f; }
  // triangulated heightfield (diagonal (i, j)-(i+1, j+1)), depth along the face normal
  const float h00 = (float)(q00 >> 8) * vs, h10 = (float)(q10 >> 8) * vs, h01 = (float)(q01 >> 8) * vs,
              h11 = (float)(q11 >> 8) * vs;
  const float fu = clampf(u - (float)i, 0.f, 1.f), fv = clampf(v - (float)j, 0.f, 1.f);
  float gx, gy, h;
  if (fu >= fv) { gx = (h10 - h00) * ihs; gy = (h11 - h10) * ihs; h = h00 + fu * (h10 - h00) + fv * (h11 - h10); }
  else          { gx = (h11 - h01) * ihs; gy = (h01 - h00) * ihs; h = h00 + fv * (h01 - h00) + fu * (h11 - h01); }
  const float inv = ph_rsqrt(gx * gx + gy * gy + 1.0f);
  *n = mk3(-gx * inv, -gy * inv, inv);
  return (h - p.z) * n->z + r;
}

// both stages for one point (the lgx_ground_contact test entry)
LGX_DEV float ground_contact(const lgx_env_params* __restrict__ P, const lgx_buffers& B, f3 p, float r, f3* n,
                             const int32_t* patch, int pi0, int pj0) {
  bool defer;
  const float d = ground_cell(P, B, p, r, n, patch, pi0, pj0, &defer);
  if (!defer) return d;
  int i, j;
  tm_cell(P, B, p, &i, &j);
  return trimesh_depth(P, B, p, r, i, j, n, patch, pi0, pj0);
}

// LDS written by some lanes of a wave and read by others of the same wave: order the accesses
// (wave-scope fences; no workgroup barrier - every queue below is wave-private)
LGX_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

#define MAX_LANE_PTS LGX_MAX_LANE_PTS
#ifndef LGX_PHYS_WAVES_PER_SIMD
#define LGX_PHYS_WAVES_PER_SIMD 1
#endif
#define HIST_STRIDE 31

// sum over the PP lanes that share a leg (lane bits 2..): contact terms were split across them
template <int PP>
LGX_DEV float psum(float v) {
  if (PP == 4) return row_quads_sum(v);   // an env is one 16-lane DPP row: two rotates
  if (PP >= 2) v += lane_xor4(v);
  if (PP >= 4) v += lane_xor8(v);
  if (PP >= 8) v += __shfl_xor(v, 16);
  return v;
}

// PP lanes per leg, 4*PP lanes per env: lane = env*4PP + p*4 + leg.  Every lane of a leg
// group computes the leg's dynamics (identical values, no extra time); the contact candidates
// of the leg are dealt round-robin over its PP lanes and their J^T W J terms reduced with
// shuffles, so the serial contact work per lane shrinks PP-fold while the chip gets PP x
// more waves (4096 envs x 16 lanes = 1024 waves for PP = 4: all 4 SIMDs of every CU busy).
template <int PP>
__global__ void __launch_bounds__(64 * PP, LGX_PHYS_WAVES_PER_SIMD)
lgx_physics_kernel(const lgx_dev_model* __restrict__ DMg, const lgx_env_params* __restrict__ P, lgx_buffers B,
                   int32_t nsub, int32_t from_actions, const float* __restrict__ act_src, int32_t frozen) {
  constexpr int PHYS_BLOCK = 64 * PP;               // 16 envs per workgroup
  constexpr int LPE = 4 * PP;                       // lanes per env
  constexpr int SLOTS = (MAX_LANE_PTS + PP - 1) / PP;
  constexpr int ENVS = 16;                          // envs per workgroup
  __shared__ lgx_dev_model smodel;                  // model tables staged once per workgroup
  __shared__ float4 slot_state[SLOTS][PHYS_BLOCK];  // per own candidate: status, fslide.xyz (lane-minor: no bank conflicts)
  // contact geometry of the candidates penetrating in pass 0 (positions do not change within a
  // substep): pass 0's classification, pass 1 and the force report read it instead of redoing
  // the frame transform and the terrain query
  __shared__ float4 geo_p[SLOTS][PHYS_BLOCK];      // contact point Pc (base-origin frame), depth
  __shared__ float4 geo_n[SLOTS][PHYS_BLOCK];      // terrain normal, candidate index
  __shared__ float hist_lds[ENVS * 4 * HIST_STRIDE];  // Go1 actuator history per (env, leg)
  // Per-leg / per-env quantities that every lane of the leg / env holds identically are kept
  // in LDS instead of VGPRs (all those lanes store the same values, so no cross-lane ordering
  // is needed): register pressure decides the occupancy of this latency-bound kernel.
  __shared__ float leg_kin[ENVS * 4][3][12];        // body frames of the leg: R (9), origin (3)
  __shared__ float leg_sys[ENVS * 4][36];           // contact-free leg system: B 18, D 6, rb 6, rl 3
  __shared__ float env_com[ENVS][40];               // base block 21, its rhs 6, base rotation 9
  // terrain around each base: height << 8 | trimesh contact-table byte (4 = unmoved, unflagged)
  __shared__ int32_t hf_patch[ENVS][LGX_HF_PATCH * LGX_HF_PATCH];
  __shared__ int32_t hf_org[ENVS][2];
  // per-wave queue of the candidates that need the corrected-trimesh query: (cells << 16 | slot << 6 | lane)
  __shared__ uint32_t tm_q[PP][64 * SLOTS];
  {
    static_assert(sizeof(lgx_dev_model) % 16 == 0, "the model is staged in 16-byte units");
    const int4* src = reinterpret_cast<const int4*>(DMg);
    int4* dst = reinterpret_cast<int4*>(&smodel);
    for (int i = threadIdx.x; i < (int)(sizeof(lgx_dev_model) / 16); i += PHYS_BLOCK) dst[i] = src[i];
    __syncthreads();
  }
  const lgx_dev_model* DM = &smodel;
  const lgx_model* M = &smodel.m;
  const int tid = threadIdx.x;
  const int gl = blockIdx.x * PHYS_BLOCK + tid;
  const int e = gl / LPE;
  const int lie = gl % LPE;
  const int eb = tid / LPE;                         // env within the workgroup
  const int leg = lie & 3;
  const int pl = lie >> 2;                          // lane index within the leg group
  const bool lane0 = leg == 0;
  const bool owner = pl == 0;                       // writes the leg's outputs
  const int N = P->num_envs;
  const bool valid = e < N;
  const int ec = valid ? e : N - 1;  // inactive lanes compute on a clamped env, never store

  LGX_CLK_DECL(12)
  const float dt = M->sim_dt;
  // ---- load state
  const float* rs = B.root_states + (int64_t)ec * 13;
  f3 pos = mk3(rs[0], rs[1], rs[2]);
  float qx = rs[3], qy = rs[4], qz = rs[5], qw = rs[6];
  f3 vlin = mk3(rs[7], rs[8], rs[9]);
  f3 wang = mk3(rs[10], rs[11], rs[12]);
  float th[3], thd[3], tgt[3], act[3];
  const float* ds = B.dof_state + (int64_t)ec * 24 + leg * 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) { th[k] = ds[2 * k]; thd[k] = ds[2 * k + 1]; }
  float mscale[4];
  mscale[0] = B.body_mass_scale[(int64_t)ec * 13];
#pragma unroll
  for (int k = 0; k < 3; ++k) mscale[1 + k] = B.body_mass_scale[(int64_t)ec * 13 + 1 + 3 * leg + k];
  const float mu = 0.5f * ((B.friction ? B.friction[ec] : 1.0f) + M->ground_friction);
  const int ctrl = P->control_type;
  const int lg = eb * 4 + leg;                      // (env, leg) slot in the workgroup
  float* hist = hist_lds + lg * HIST_STRIDE;
  float* kin = &leg_kin[lg][0][0];
  float* lsys = leg_sys[lg];
  float* ecom = env_com[eb];
  const bool use_hist = from_actions && P->use_actuator_history;
  if (from_actions) {  // clip (legged_robot.py:85-86) fused into the load
    const float* a = act_src + (int64_t)ec * 12 + leg * 3;  // raw actions (B.actions or lgx_step_from's input)
#pragma unroll
    for (int k = 0; k < 3; ++k) act[k] = clampf(a[k], -P->clip_actions, P->clip_actions);
  }
  if (ctrl == LGX_CTRL_POS_DRIVE) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      int j = 3 * leg + k;
      // _compute_poses (legged_robot.py:394-397); identical every substep
      tgt[k] = from_actions ? clampf(act[k] * P->action_scale + P->default_dof_pos[j], P->soft_lower[j], P->soft_upper[j])
                            : B.dof_targets[(int64_t)ec * 12 + j];
    }
  }
  if (use_hist) {
    const float* h = B.act_hist + (int64_t)ec * 120 + leg * 30;
#pragma unroll
    for (int i = 0; i < 30; ++i) hist[i] = h[i];
  }
  // heightfield patch of each env (rough terrain): LGX_HF_PATCH^2 samples centred on the base at
  // the start of the launch; contact queries inside it read LDS instead of gathering from HBM
  const bool use_patch = P->terrain_kind != 0 && B.height_samples != nullptr && B.hf_rows >= LGX_HF_PATCH &&
                         B.hf_cols >= LGX_HF_PATCH;
  if (use_patch) {
    if (lie == 0) {
      const float hs = P->horizontal_scale;
      int ci = (int)floorf((pos.x + P->border_size) / hs), cj = (int)floorf((pos.y + P->border_size) / hs);
      hf_org[eb][0] = min(max(ci - LGX_HF_PATCH / 2, 0), B.hf_rows - LGX_HF_PATCH);
      hf_org[eb][1] = min(max(cj - LGX_HF_PATCH / 2, 0), B.hf_cols - LGX_HF_PATCH);
    }
    __syncthreads();
    // every thread copies PER samples, in batches of up to 12 whose global loads are all issued
    // before the first LDS store (the copy is latency-bound otherwise: one HBM round trip per sample)
    constexpr int AREA = LGX_HF_PATCH * LGX_HF_PATCH, PER = ENVS * AREA / PHYS_BLOCK;
    constexpr int BATCH = PER % 12 == 0 ? 12 : PER % 9 == 0 ? 9 : PER % 8 == 0 ? 8 : PER % 6 == 0 ? 6 : 4;
    static_assert(ENVS * AREA % PHYS_BLOCK == 0 && PER % BATCH == 0, "patch copy layout");
    const int8_t* T = B.hf_trimesh;
    for (int q0 = 0; q0 < PER; q0 += BATCH) {
      int16_t hv[BATCH];
      int8_t tv[BATCH];
#pragma unroll
      for (int b = 0; b < BATCH; ++b) {
        const int q = tid + (q0 + b) * PHYS_BLOCK;
        const int ee = q / AREA, r = q % AREA;
        const int64_t gi = (int64_t)(hf_org[ee][0] + r / LGX_HF_PATCH) * B.hf_cols + hf_org[ee][1] + r % LGX_HF_PATCH;
        hv[b] = B.height_samples[gi];
        tv[b] = T ? T[gi] : (int8_t)4;
      }
#pragma unroll
      for (int b = 0; b < BATCH; ++b) {
        const int q = tid + (q0 + b) * PHYS_BLOCK;
        hf_patch[q / AREA][q % AREA] = ((int32_t)hv[b] << 8) | (tv[b] & 0xff);
      }
    }
    __syncthreads();
  }
  const int32_t* patch = use_patch ? hf_patch[eb] : nullptr;
  const int pi0 = use_patch ? hf_org[eb][0] : 0, pj0 = use_patch ? hf_org[eb][1] : 0;
  const int npts = DM->lane_npts[leg];
  const int maxpts = DM->max_lane_npts;
  const bool rot_eye = __builtin_amdgcn_readfirstlane(DM->joint_rot_eye) != 0;   // uniform
  // this lane's candidates (point index, dynamic body) per slot, fixed for the launch: the geometry
  // loop's model reads then no longer wait on one another
  int slot_pt[SLOTS], slot_db[SLOTS];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) {
    const int c = pl + PP * sl;
    slot_pt[sl] = DM->lane_pts[leg][c < npts ? c : 0];
    slot_db[sl] = M->point_dyn[slot_pt[sl]];
  }
  f3 cf_leg[4] = {mk3(0, 0, 0), mk3(0, 0, 0), mk3(0, 0, 0), mk3(0, 0, 0)};
  f3 cf_base = mk3(0, 0, 0);
  float tq[3] = {0.f, 0.f, 0.f};

  LGX_CLK(6);
  for (int s = 0; s < nsub; ++s) {
    // ---- Go1 actuator-net history (go1.py:79-98), model_ins per substep
    if (use_hist) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        int j = 3 * leg + k;
        float pe = act[k] - th[k];
        float pes = (pe - P->act_pos_err_mean[j]) / P->act_pos_err_std[j];
        float vs = (thd[k] - P->act_vel_mean[j]) / P->act_vel_std[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) { hist[10 * k + i] = hist[10 * k + i + 1]; hist[10 * k + 5 + i] = hist[10 * k + 6 + i]; }
        hist[10 * k + 4] = pes;
        hist[10 * k + 9] = vs;
      }
      if (valid && owner) {
        float* mi = B.model_ins + ((int64_t)s * N + e) * 120 + leg * 30;
#pragma unroll
        for (int i = 0; i < 30; i += 2) *reinterpret_cast<float2*>(mi + i) = make_float2(hist[i], hist[i + 1]);
      }
    }
    // ---- explicit-torque controllers (_compute_torques, legged_robot.py:370-392)
    float tex[3] = {0.f, 0.f, 0.f};
    if (ctrl != LGX_CTRL_POS_DRIVE && !from_actions) {
#pragma unroll
      for (int k = 0; k < 3; ++k) tex[k] = B.torques[(int64_t)ec * 12 + 3 * leg + k];  // caller-provided torques
    } else if (ctrl == LGX_CTRL_SEA) {
      // the leg's 3 joints dealt over its PP lanes (joint k on lane p = k % PP, pass k / PP), then
      // every lane of the leg takes the 3 torques by shuffle; clamped to the drive's effort limit
      // (PhysX DOF effort mode, URDF effort)
      constexpr int PASSES = (3 + PP - 1) / PP;
      float mine[PASSES];
      const int64_t m = (int64_t)N * 12;
#pragma unroll
      for (int q = 0; q < PASSES; ++q) {
        const int kk = pl + q * PP;
        const int k = kk < 3 ? kk : 2;
        const float a = k == 0 ? act[0] : (k == 1 ? act[1] : act[2]);
        const float qq = k == 0 ? th[0] : (k == 1 ? th[1] : th[2]);
        const float qd = k == 0 ? thd[0] : (k == 1 ? thd[1] : thd[2]);
        const int j = 3 * leg + k;
        mine[q] = sea_lstm(B.sea_w, B.sea_h, B.sea_c, (int64_t)ec * 12 + j, m,
                           a * P->action_scale + P->default_dof_pos[j] - qq, qd, valid && kk < 3);
      }
      const int base = (threadIdx.x & 63) - 4 * pl;   // this leg's lane p = 0 in the wave
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float t = PP == 1 ? mine[k] : __shfl(mine[k / PP], base + 4 * (k % PP), 64);
        const float eff = M->dof_effort[3 * leg + k];
        tex[k] = clampf(t, -eff, eff);
      }
    } else if (ctrl != LGX_CTRL_POS_DRIVE) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        int j = 3 * leg + k;
        float a = act[k] * P->action_scale, t;
        if (ctrl == LGX_CTRL_P) t = P->p_gains[j] * (a + P->default_dof_pos[j] - th[k]) - P->d_gains[j] * thd[k];
        else if (ctrl == LGX_CTRL_V)
          t = P->p_gains[j] * (a - thd[k]) - P->d_gains[j] * (thd[k] - B.last_dof_vel[(int64_t)ec * 12 + j]) / dt;
        else t = a;
        tex[k] = clampf(t, -P->torque_limits[j], P->torque_limits[j]);
      }
    }
    LGX_CLK(0);
    // frozen (lgx_drive_inputs): the drive inputs above - clipped actions, targets, actuator-net
    // history / model_ins rows, SEA LSTM state and torques - with the physical state held fixed,
    // no dynamics (uniform branch)
    if (frozen) {
      if (ctrl == LGX_CTRL_SEA) { tq[0] = tex[0]; tq[1] = tex[1]; tq[2] = tex[2]; }
      continue;
    }
    // ---- kinematics
    m33 R0 = quat_to_mat(qx, qy, qz, qw);
    m33 Rb[3];
    f3 ob[3];
    sv S[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) ecom[27 + i] = R0.a[i];
    ecom[36] = pos.x; ecom[37] = pos.y; ecom[38] = pos.z;
    {
      m33 Rp = R0;
      f3 op = mk3(0, 0, 0);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        int j = 3 * leg + k;
        m33 Rjf = Rp;   // identity joint frames (every quadruped but ANYmal C): no R_p E product
        if (!rot_eye) {
          m33 E;
#pragma unroll
          for (int i = 0; i < 9; ++i) E.a[i] = M->joint_rot[j][i];
          Rjf = mul(Rp, E);
        }
        f3 oj = op + mul(Rp, mk3(M->joint_pos[j][0], M->joint_pos[j][1], M->joint_pos[j][2]));
        f3 ax = mk3(M->joint_axis[j][0], M->joint_axis[j][1], M->joint_axis[j][2]);
        f3 aw = mul(Rjf, ax);
#if LGX_PHYS_FAST_TRANSC
        Rb[k] = mul(Rjf, axis_angle_hw(ax, th[k]));
#else
        Rb[k] = mul(Rjf, axis_angle(ax, th[k]));
#endif
        ob[k] = oj;
#pragma unroll
        for (int i = 0; i < 9; ++i) kin[k * 12 + i] = Rb[k].a[i];
        kin[k * 12 + 9] = oj.x; kin[k * 12 + 10] = oj.y; kin[k * 12 + 11] = oj.z;
        S[k] = sv{aw, cross(oj, aw)};
        Rp = Rb[k];
        op = oj;
      }
    }
    SI Ibase = body_si(M, 0, mscale[0], R0, mk3(0, 0, 0));
    SI Il[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Il[k] = body_si(M, 1 + 3 * leg + k, mscale[1 + k], Rb[k], ob[k]);
    // ---- RNEA bias forces, A_0 = (0, -w x v - g)
    sv V0 = sv{wang, vlin};
    sv A0 = sv{mk3(0, 0, 0), mk3(0, 0, 0) - cross(wang, vlin) - mk3(M->gravity[0], M->gravity[1], M->gravity[2])};
    sv Vk[3], fk[3];
    {
      sv Vp = V0, Ap = A0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sv V = add(Vp, scale(thd[k], S[k]));
        sv A = add(Ap, scale(thd[k], crm(V, S[k])));
        fk[k] = add(si_mul(Il[k], A), crf(V, si_mul(Il[k], V)));
        Vk[k] = V;
        Vp = V; Ap = A;
      }
    }
    sv F2 = fk[2], F1 = add(fk[1], F2), F0 = add(fk[0], F1);
    float Cl[3] = {dot(S[0], F0), dot(S[1], F1), dot(S[2], F2)};
    sv fbase = add(si_mul(Ibase, A0), crf(V0, si_mul(Ibase, V0)));
    // ---- CRBA: composite inertias, B = [IC_k S_k], D_kk' = S_k . IC_k' S_k'
    SI IC2 = Il[2], IC1 = si_add(Il[1], IC2), IC0 = si_add(Il[0], IC1);
    sv Fc[3] = {si_mul(IC0, S[0]), si_mul(IC1, S[1]), si_mul(IC2, S[2])};
    LegSys L0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int k = 0; k < 3; ++k) L0.B[i][k] = sv_get(Fc[k], i);
    L0.D[0] = dot(S[0], Fc[0]); L0.D[1] = dot(S[1], Fc[1]); L0.D[2] = dot(S[2], Fc[2]);
    L0.D[3] = dot(S[0], Fc[1]); L0.D[4] = dot(S[0], Fc[2]); L0.D[5] = dot(S[1], Fc[2]);
    // base block common part: total composite inertia (quad-reduced)
    float Acom[21];
    {
      SI tot = IC0;
      tot.m = quad_sum(tot.m);
      tot.h = mk3(quad_sum(tot.h.x), quad_sum(tot.h.y), quad_sum(tot.h.z));
#pragma unroll
      for (int i = 0; i < 6; ++i) tot.I[i] = quad_sum(tot.I[i]);
      tot = si_add(tot, Ibase);
      si_to_sym6(tot, Acom);
    }
#pragma unroll
    for (int i = 0; i < 21; ++i) ecom[i] = Acom[i];
    // H u and bias: rb = A u_b - dt f_base + sum_l (B_l qd_l - dt F0_l);  rl = B^T u_b + D qd + dt(g - C)
    float ub[6] = {wang.x, wang.y, wang.z, vlin.x, vlin.y, vlin.z};
    float rbcom[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      float s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 6; ++j) s2 += Acom[sidx(i, j)] * ub[j];
      rbcom[i] = s2 - dt * sv_get(fbase, i);
      ecom[21 + i] = rbcom[i];
    }
    float rb0[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rb0[i] = L0.B[i][0] * thd[0] + L0.B[i][1] * thd[1] + L0.B[i][2] * thd[2] - dt * sv_get(F0, i);
    float rl0[3];
    {
      f3 Dq = sym3_mul(L0.D, mk3(thd[0], thd[1], thd[2]));
      float dqv[3] = {Dq.x, Dq.y, Dq.z};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 6; ++i) s2 += L0.B[i][k] * ub[i];
        rl0[k] = s2 + dqv[k] - dt * Cl[k];
      }
    }
    LGX_CLK(1);
    // ---- drives and limits
    float Dimp[3] = {0.f, 0.f, 0.f};
    bool impl[3] = {false, false, false};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      int j = 3 * leg + k;
      // model reads first (LDS): a read inside a lane-dependent branch waits on its own round trip
      const float kp = M->kp[j], kd = M->kd[j], eff = M->dof_effort[j];
      const float lo = M->dof_lower[j], hi = M->dof_upper[j], lk = M->limit_k, lc = M->limit_c;
      float g = 0.f;
      if (ctrl == LGX_CTRL_POS_DRIVE) {
        float te = kp * (tgt[k] - th[k]) - kd * thd[k];
        if (fabsf(te) <= eff) {
          impl[k] = true;
          Dimp[k] += dt * (kd + dt * kp);
          g += kp * (tgt[k] - th[k]);
        } else {
          g += te > 0.f ? eff : -eff;
        }
      } else {
        g += tex[k];
      }
      if (lo < hi) {
        if (th[k] < lo) { Dimp[k] += dt * (lc + dt * lk); g += lk * (lo - th[k]); }
        else if (th[k] > hi) { Dimp[k] += dt * (lc + dt * lk); g -= lk * (th[k] - hi); }
      }
      rl0[k] += dt * g;
    }
    L0.D[0] += Dimp[0]; L0.D[1] += Dimp[1]; L0.D[2] += Dimp[2];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      lsys[3 * i] = L0.B[i][0]; lsys[3 * i + 1] = L0.B[i][1]; lsys[3 * i + 2] = L0.B[i][2];
      lsys[18 + i] = L0.D[i];
      lsys[24 + i] = rb0[i];
    }
    lsys[30] = rl0[0]; lsys[31] = rl0[1]; lsys[32] = rl0[2];
    LGX_CLK(2);
    // ---- contacts: two passes (pass 0 implicit stick, pass 1 with slide / drop decisions)
    const float kn = M->contact_k, cn = M->contact_c, ct = M->friction_c;
    const float wn = dt * (cn + dt * kn);
    // contact geometry of every candidate (positions do not change within the substep): contact
    // point, depth and normal of the penetrating ones into LDS, before any contact term is formed
    // (the terrain queries run without the 54 accumulator registers live).  The corrected-trimesh
    // query is rare and long: a wave would run it once for every slot in which any of its lanes
    // needs it, so those candidates are queued (wave-private, ballot-compacted) and answered
    // afterwards 64 at a time - first the block-height test that dismisses the spheres high above
    // the ground, then the full query for the near ones.  Same arithmetic per candidate.
    {
      const int ln = tid & 63, wv = tid >> 6;
      const uint64_t below = (1ull << ln) - 1;
      const int nslots = (maxpts + PP - 1) / PP;    // wave-uniform slot count
      int qn = 0;
#pragma unroll
      for (int sl = 0; sl < SLOTS; ++sl) {
        if (sl >= nslots) break;
        const bool act = pl + PP * sl < npts;
        const int pi = slot_pt[sl];
        const int db = slot_db[sl];
        const int k = db == 0 ? -1 : (db - 1) % 3;
        const float* fr = db == 0 ? ecom + 27 : kin + 12 * k;   // body rotation (+ origin) in LDS
        m33 R;
#pragma unroll
        for (int i = 0; i < 9; ++i) R.a[i] = fr[i];
        f3 ol = db == 0 ? mk3(0, 0, 0) : mk3(fr[9], fr[10], fr[11]);
        f3 Pp = ol + mul(R, mk3(M->point_pos[pi][0], M->point_pos[pi][1], M->point_pos[pi][2]));
        const float rad = M->point_radius[pi];
        f3 n;
        bool defer;
        const float depth = ground_cell(P, B, Pp + pos, rad, &n, patch, pi0, pj0, &defer);
        defer = defer && act;
        const uint64_t m = __ballot(defer);
        if (defer) {
          tm_q[wv][qn + __popcll(m & below)] = (uint32_t)(sl << 6 | ln);
          geo_p[sl][tid] = make_float4(Pp.x, Pp.y, Pp.z, rad);
          geo_n[sl][tid] = make_float4(0.f, 0.f, 1.f, (float)pi);
        } else if (act) {
          slot_state[sl][tid] = make_float4(depth > 0.f ? 1.f : 0.f, 0.f, 0.f, 0.f);
          if (depth > 0.f) {
            const f3 Pc = Pp - rad * n;
            geo_p[sl][tid] = make_float4(Pc.x, Pc.y, Pc.z, depth);
            geo_n[sl][tid] = make_float4(n.x, n.y, n.z, (float)pi);
          }
        }
        qn += __popcll(m);
      }
      LGX_CLK(8);
      if (qn > 0) {
        wave_lds_sync();
        // stage 1: which cells of the 3 x 3 each sphere has to visit, survivors compacted in place with
        // their cell set (a round reads all its entries before it writes any, and writes only
        // positions below the ones it read).  Short queues (a Go1's feet): the block-height test
        // alone (the spheres well above the ground leave), every cell kept - stage 2 culls them per
        // lane; long queues (a capsule-covered robot like ANYmal on stairs): the cell culls too, so
        // fewer spheres reach stage 2 and each visits only its kept cells
        const bool cull1 = qn > 16;
        int qn2 = 0;
        for (int q0 = 0; q0 < qn; q0 += 64) {
          const int q = q0 + ln;
          uint32_t ent = 0;
          unsigned keep = 0;
          if (q < qn) {
            ent = tm_q[wv][q];
            const int sl2 = (ent >> 6) & 1023, t = (wv << 6) | (ent & 63), e2 = t / LPE;
            const float4 g = geo_p[sl2][t];
            const f3 pw = mk3(g.x, g.y, g.z) + mk3(env_com[e2][36], env_com[e2][37], env_com[e2][38]);
            const int32_t* hp = use_patch ? hf_patch[e2] : nullptr;
            const int o0 = use_patch ? hf_org[e2][0] : 0, o1 = use_patch ? hf_org[e2][1] : 0;
            int i, j;
            tm_cell(P, B, pw, &i, &j);
            if (cull1) {
              f3 pl3;
              keep = tm_keep(P, B, pw, g.w, i, j, hp, o0, o1, &pl3);
            } else {
              keep = tm_near(P, B, pw, g.w, i, j, hp, o0, o1) ? 0x1ffu : 0u;
            }
            if (!keep) slot_state[sl2][t] = make_float4(0.f, 0.f, 0.f, 0.f);
          }
          const uint64_t m = __ballot(keep != 0);
          if (keep) tm_q[wv][qn2 + __popcll(m & below)] = ent | keep << 16;
          qn2 += __popcll(m);
        }
        wave_lds_sync();
        LGX_CLK(9);
#ifdef LGX_PHASE_CLOCK
        lgx_clk_acc[11] += (uint64_t)qn * 1000 + qn2;   // queue lengths (tuning builds)
#endif
        // stage 2: the kept cells of each near sphere.  Few spheres (the common case: a robot's feet on
        // a riser): 16 lanes per sphere, lane g < 9 of the row visits cell g if kept, the row combines
        // in the sequential scan's order.  Many (a capsule-covered robot like ANYmal on stairs): one
        // lane per sphere visiting its kept cells in order (a round costs its lane with the most
        // cells, typically 1 - 3 of the 9)
        if (qn2 <= 8) {
          const int grp = ln >> 4, g = ln & 15;
          for (int q0 = 0; q0 < qn2; q0 += 4) {
            const int q = min(q0 + grp, qn2 - 1);
            const uint32_t ent = tm_q[wv][q];
            const int sl2 = (ent >> 6) & 1023, t = (wv << 6) | (ent & 63), e2 = t / LPE;
            const float4 gp = geo_p[sl2][t];
            const f3 Pp = mk3(gp.x, gp.y, gp.z);
            const f3 pw = Pp + mk3(env_com[e2][36], env_com[e2][37], env_com[e2][38]);
            const int32_t* hp = use_patch ? hf_patch[e2] : nullptr;
            const int o0 = use_patch ? hf_org[e2][0] : 0, o1 = use_patch ? hf_org[e2][1] : 0;
            int i, j;
            tm_cell(P, B, pw, &i, &j);
            const f3 pl3 = tm_local(P, pw, i, j);
            TmQuery tq;
            tm_init(tq, pl3);
            if (g < 9 && ((ent >> (16 + g)) & 1u))
              tm_cell_tris(tq, P, B, pl3, gp.w, i, j, (g * 11) >> 5, g - 3 * ((g * 11) >> 5), hp, o0, o1);
            int cd2 = g, ctop = g;
            tm_combine_step<1>(tq, cd2, ctop);
            tm_combine_step<2>(tq, cd2, ctop);
            tm_combine_step<4>(tq, cd2, ctop);
            tm_combine_step<8>(tq, cd2, ctop);
            if (g == 0 && q0 + grp < qn2) {
              f3 n;
              const float depth = tm_finish(tq, pl3, gp.w, &n);
              slot_state[sl2][t] = make_float4(depth > 0.f ? 1.f : 0.f, 0.f, 0.f, 0.f);
              if (depth > 0.f) {
                const f3 Pc = Pp - gp.w * n;
                geo_p[sl2][t] = make_float4(Pc.x, Pc.y, Pc.z, depth);
                geo_n[sl2][t] = make_float4(n.x, n.y, n.z, geo_n[sl2][t].w);
              }
            }
          }
        } else {
          for (int q0 = 0; q0 < qn2; q0 += 64) {
            const int q = q0 + ln;
            if (q < qn2) {
              const uint32_t ent = tm_q[wv][q];
              const int sl2 = (ent >> 6) & 1023, t = (wv << 6) | (ent & 63), e2 = t / LPE;
              const float4 gp = geo_p[sl2][t];
              const f3 Pp = mk3(gp.x, gp.y, gp.z);
              const f3 pw = Pp + mk3(env_com[e2][36], env_com[e2][37], env_com[e2][38]);
              int i, j;
              tm_cell(P, B, pw, &i, &j);
              f3 n;
              const float depth = tm_visit(P, B, tm_local(P, pw, i, j), gp.w, i, j, ent >> 16, &n,
                                           use_patch ? hf_patch[e2] : nullptr, use_patch ? hf_org[e2][0] : 0,
                                           use_patch ? hf_org[e2][1] : 0);
              slot_state[sl2][t] = make_float4(depth > 0.f ? 1.f : 0.f, 0.f, 0.f, 0.f);
              if (depth > 0.f) {
                const f3 Pc = Pp - gp.w * n;
                geo_p[sl2][t] = make_float4(Pc.x, Pc.y, Pc.z, depth);
                geo_n[sl2][t] = make_float4(n.x, n.y, n.z, geo_n[sl2][t].w);
              }
            }
          }
        }
      }
      wave_lds_sync();
    }
    LGX_CLK(10);
    float xb[6];
    f3 xl;
    for (int pass = 0; pass < 2; ++pass) {
      LegSys L;  // this lane's contact terms
#pragma unroll
      for (int i = 0; i < 21; ++i) L.Ap[i] = 0.f;
#pragma unroll
      for (int i = 0; i < 6; ++i) { L.rb[i] = 0.f; L.B[i][0] = L.B[i][1] = L.B[i][2] = 0.f; }
#pragma unroll
      for (int i = 0; i < 6; ++i) L.D[i] = 0.f;
      L.rl[0] = L.rl[1] = L.rl[2] = 0.f;
      for (int c = pl, sl = 0; c < maxpts; c += PP, ++sl) {
        if (c >= npts) break;
        const float4 st = slot_state[sl][tid];
        if (st.x == 0.f) continue;  // separated (pass 1: in pass 0's classification)
        const float4 gp = geo_p[sl][tid], gn = geo_n[sl][tid];
        const f3 Pc = mk3(gp.x, gp.y, gp.z);
        const float depth = gp.w;
        const f3 n = mk3(gn.x, gn.y, gn.z);
        const int db = M->point_dyn[(int)gn.w];
        const int k = db == 0 ? -1 : (db - 1) % 3;
        float wt = (pass == 0 || st.x == 1.f) ? dt * ct : 0.f;
        f3 f = (dt * kn * depth) * n;
        if (pass == 1 && st.x == 2.f) f = f + dt * mk3(st.y, st.z, st.w);
        add_contact(L, Pc, n, wn, wt, f, k, S);
      }
      // reduce the contact terms over the PP lanes of the leg, add the contact-free system
#pragma unroll
      for (int i = 0; i < 21; ++i) L.Ap[i] = psum<PP>(L.Ap[i]);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        L.rb[i] = psum<PP>(L.rb[i]) + lsys[24 + i];
#pragma unroll
        for (int k = 0; k < 3; ++k) L.B[i][k] = psum<PP>(L.B[i][k]) + lsys[3 * i + k];
        L.D[i] = psum<PP>(L.D[i]) + lsys[18 + i];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) L.rl[k] = psum<PP>(L.rl[k]) + lsys[30 + k];
      if (pass == 0) LGX_CLK(3); else LGX_CLK(7);
      arrow_solve(L, ecom, ecom + 21, lane0, xb, xl);
      LGX_CLK(4);
      // contact status (after pass 0) / reported forces (after pass 1, last substep)
      const bool report = pass == 1 && s == nsub - 1;
      if (pass == 0 || report) {
        sv Vb = sv{mk3(xb[0], xb[1], xb[2]), mk3(xb[3], xb[4], xb[5])};
        sv Vl[3];
        Vl[0] = add(Vb, scale(xl.x, S[0]));
        Vl[1] = add(Vl[0], scale(xl.y, S[1]));
        Vl[2] = add(Vl[1], scale(xl.z, S[2]));
        for (int c = pl, sl = 0; c < maxpts; c += PP, ++sl) {
          if (c >= npts) break;
          float4 st = slot_state[sl][tid];
          if (st.x == 0.f) continue;
          const float4 gp = geo_p[sl][tid], gn = geo_n[sl][tid];
          const f3 Pc = mk3(gp.x, gp.y, gp.z), n = mk3(gn.x, gn.y, gn.z);
          const float depth = gp.w;
          const int pi = (int)gn.w;
          const int db = M->point_dyn[pi];
          const int k = db == 0 ? -1 : (db - 1) % 3;
          sv V = db == 0 ? Vb : sel3(k, Vl[0], Vl[1], Vl[2]);
          f3 vp = V.l + cross(V.a, Pc);
          float vn = dot(vp, n);
          float fn = kn * depth - (cn + dt * kn) * vn;
          f3 vt = vp - vn * n;
          if (pass == 0) {
            float vtn = sqrtf(dot(vt, vt));
            if (fn <= 0.f) st.x = 0.f;
            else if (ct * vtn > mu * fn) {
              float sc = -mu * fn / vtn;
              st = make_float4(2.f, sc * vt.x, sc * vt.y, sc * vt.z);
            } else st.x = 1.f;
            slot_state[sl][tid] = st;
          } else {
            fn = fmaxf(fn, 0.f);
            f3 ft = st.x == 1.f ? (-ct) * vt : mk3(st.y, st.z, st.w);
            f3 F = fn * n + ft;
            int rep = M->point_report[pi];
            if (rep == 0) cf_base = cf_base + F;
            else {
              int r = rep - (1 + 4 * leg);
              cf_leg[0] = r == 0 ? cf_leg[0] + F : cf_leg[0];
              cf_leg[1] = r == 1 ? cf_leg[1] + F : cf_leg[1];
              cf_leg[2] = r == 2 ? cf_leg[2] + F : cf_leg[2];
              cf_leg[3] = r == 3 ? cf_leg[3] + F : cf_leg[3];
            }
          }
        }
      }
      LGX_CLK(5);  // classification / reporting
    }
    // ---- joint outputs and integration
    float qdn[3] = {xl.x, xl.y, xl.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      int j = 3 * leg + k;
      float q2 = qdn[k];
      float vl = M->dof_vel_limit[j];
      if (vl > 0.f) q2 = clampf(q2, -vl, vl);
      if (ctrl == LGX_CTRL_POS_DRIVE) {
        float eff = M->dof_effort[j];
        float t = impl[k] ? M->kp[j] * (tgt[k] - th[k] - dt * qdn[k]) - M->kd[j] * qdn[k]
                          : M->kp[j] * (tgt[k] - th[k]) - M->kd[j] * thd[k];
        tq[k] = clampf(t, -eff, eff);
      } else {
        tq[k] = tex[k];
      }
      th[k] = th[k] + dt * q2;
      thd[k] = q2;
    }
    wang = mk3(xb[0], xb[1], xb[2]);
    vlin = mk3(xb[3], xb[4], xb[5]);
    pos = pos + dt * vlin;
    {
      f3 qv = mk3(qx, qy, qz);
      f3 wq = cross(wang, qv);
      float dqx = 0.5f * (qw * wang.x + wq.x), dqy = 0.5f * (qw * wang.y + wq.y), dqz = 0.5f * (qw * wang.z + wq.z);
      float dqw = -0.5f * dot(wang, qv);
      qx += dt * dqx; qy += dt * dqy; qz += dt * dqz; qw += dt * dqw;
      float inv = 1.0f / sqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
      qx *= inv; qy *= inv; qz *= inv; qw *= inv;
    }
  }

  // ---- write back
  cf_base = mk3(psum<PP>(quad_sum(cf_base.x)), psum<PP>(quad_sum(cf_base.y)), psum<PP>(quad_sum(cf_base.z)));
#pragma unroll
  for (int r = 0; r < 4; ++r) cf_leg[r] = mk3(psum<PP>(cf_leg[r].x), psum<PP>(cf_leg[r].y), psum<PP>(cf_leg[r].z));
  if (!valid || !owner) return;
  if (from_actions) {
    float* ao = B.actions + (int64_t)e * 12 + leg * 3;
    ao[0] = act[0]; ao[1] = act[1]; ao[2] = act[2];
  }
  if (frozen) {
    if (ctrl == LGX_CTRL_POS_DRIVE && from_actions) {
      float* to = B.dof_targets + (int64_t)e * 12 + leg * 3;
      to[0] = tgt[0]; to[1] = tgt[1]; to[2] = tgt[2];
    }
    if (use_hist) {
      float* h = B.act_hist + (int64_t)e * 120 + leg * 30;
#pragma unroll
      for (int i = 0; i < 30; i += 2) *reinterpret_cast<float2*>(h + i) = make_float2(hist[i], hist[i + 1]);
    }
    if (ctrl == LGX_CTRL_SEA && from_actions && nsub > 0) {   // the last substep's network torques
      float* tqo = B.torques + (int64_t)e * 12 + leg * 3;
      tqo[0] = tq[0]; tqo[1] = tq[1]; tqo[2] = tq[2];
    }
    return;
  }
  float* dso = B.dof_state + (int64_t)e * 24 + leg * 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) *reinterpret_cast<float2*>(dso + 2 * k) = make_float2(th[k], thd[k]);
  float* tqo = B.torques + (int64_t)e * 12 + leg * 3;
  if (nsub > 0) { tqo[0] = tq[0]; tqo[1] = tq[1]; tqo[2] = tq[2]; }
  if (ctrl == LGX_CTRL_POS_DRIVE && from_actions) {
    float* to = B.dof_targets + (int64_t)e * 12 + leg * 3;
    to[0] = tgt[0]; to[1] = tgt[1]; to[2] = tgt[2];
  }
  float* cfo = B.contact_forces + (int64_t)e * LGX_MAX_BODIES * 3;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* d = cfo + (1 + 4 * leg + r) * 3;
    d[0] = cf_leg[r].x; d[1] = cf_leg[r].y; d[2] = cf_leg[r].z;
  }
  if (use_hist) {
    float* h = B.act_hist + (int64_t)e * 120 + leg * 30;
#pragma unroll
    for (int i = 0; i < 30; i += 2) *reinterpret_cast<float2*>(h + i) = make_float2(hist[i], hist[i + 1]);
  }
  if (lane0) {
    cfo[0] = cf_base.x; cfo[1] = cf_base.y; cfo[2] = cf_base.z;
    float* ro = B.root_states + (int64_t)e * 13;
    ro[0] = pos.x; ro[1] = pos.y; ro[2] = pos.z;
    ro[3] = qx; ro[4] = qy; ro[5] = qz; ro[6] = qw;
    ro[7] = vlin.x; ro[8] = vlin.y; ro[9] = vlin.z;
    ro[10] = wang.x; ro[11] = wang.y; ro[12] = wang.z;
  }
  LGX_CLK(7);
  LGX_CLK_PRINT("physics", 12)
}

// ground_contact for a batch of world points (test entry lgx_ground_contact): q[k] = (x, y, z, r)
// -> o[k] = (depth, nx, ny, nz); heights / table read from global memory (no LDS patch)
__global__ void lgx_ground_contact_kernel(const lgx_env_params* __restrict__ P, lgx_buffers B, const float4* __restrict__ q,
                                          int32_t n, float4* __restrict__ o) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float4 v = q[k];
  f3 nn;
  const float d = ground_contact(P, B, mk3(v.x, v.y, v.z), v.w, &nn, nullptr, 0, 0);
  o[k] = make_float4(d, nn.x, nn.y, nn.z);
}

int lgx_launch_ground_contact(const lgx_env_params* dp, const lgx_buffers& b, const float* q, int32_t n, float* o,
                              hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(lgx_ground_contact_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, dp, b,
                     reinterpret_cast<const float4*>(q), n, reinterpret_cast<float4*>(o));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// lanes per leg: 4 at every size (4096 envs x 16 lanes = 1024 waves = one per SIMD; larger batches run
// in rounds of one 16-env workgroup per CU - the 148 KB of LDS per workgroup admit one, so a 2- or
// 1-lane split would leave 2 or 3 SIMDs of each CU idle: measured C5 8192 envs 355 -> 283 us,
// 16384 envs 670 -> 568 us for 2 -> 4 lanes); LGX_PHYS_PP (1, 2, 4, 8) overrides it for A/B runs
// and for the parity tests of every split
int lgx_physics_pp(int32_t n_envs) {
  (void)n_envs;
  const char* force = getenv("LGX_PHYS_PP");
  const int f = force ? atoi(force) : 0;
  return (f == 1 || f == 2 || f == 4 || f == 8) ? f : 4;
}

int lgx_launch_physics(const lgx_dev_model* dm, const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs,
                       int32_t nsub, int32_t from_actions, const float* act_src, hipStream_t stream, int32_t frozen,
                       int ppx) {
  if (!act_src) act_src = b.actions;
  const int blocks = (n_envs + 15) / 16;       // 16 envs per workgroup of 64*PP lanes
  if (ppx == 8)
    LGX_LAUNCH(lgx_physics_kernel<8>, dim3(blocks), dim3(512), 0, stream, dm, dp, b, nsub, from_actions, act_src, frozen);
  else if (ppx == 4)
    LGX_LAUNCH(lgx_physics_kernel<4>, dim3(blocks), dim3(256), 0, stream, dm, dp, b, nsub, from_actions, act_src, frozen);
  else if (ppx == 2)
    LGX_LAUNCH(lgx_physics_kernel<2>, dim3(blocks), dim3(128), 0, stream, dm, dp, b, nsub, from_actions, act_src, frozen);
  else
    LGX_LAUNCH(lgx_physics_kernel<1>, dim3(blocks), dim3(64), 0, stream, dm, dp, b, nsub, from_actions, act_src, frozen);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


// ============================================================================================
// Dense joint-space physics (lgx_model.leg_dof == 6: Cassie's 2 legs x 6 joints, which the
// arrowhead kernel's 4-leg x 3-joint lane mapping does not cover; any robot with LGX_PHYS_DENSE=1).
// One env per wavefront (64-thread workgroup), the same physics model as the oracle (implicit PD
// drives and limit springs, compliant contact with the two-pass stick / slide classification) on the
// full 18 x 18 joint-space system, the work of every phase spread over the wave's lanes with the
// per-env arrays in LDS:
//   * one lane per leg chain: forward kinematics and the RNEA velocities / accelerations on the way
//     out, then composite inertias IC_k, H's leg rows (S_j . IC_k S_k) and base couplings (IC_k S_k),
//     and the bias forces S_j . (sum of the subtree's body forces) on the way back (CRBA / RNEA: the
//     H = sum_b J_b^T I_b J_b of the oracle without its zero blocks);
//   * one lane per body: spatial inertia and body force; one lane per entry: the base block;
//   * one lane per contact candidate (ballot-compacted in point order, so the sums over contacts run
//     in the oracle's order); one lane per matrix entry of M = H + drives + contact terms; one lane
//     per row in each Cholesky column.
// Contact storage is sized to the robot's candidate count (dynamic LDS).  Latency-bound like the
// arrowhead kernel (a serial chain of small dependent steps per env).
// ============================================================================================
namespace {

constexpr int DN = 18;                     // generalised velocity [w(3), v(3), qd(12)]
constexpr int DCF = 3 * DN + 3 + 3 + 1 + 1 + 3 + 3;   // floats per contact slot (+ 3 ints)

struct DenseLds {
  float R[LGX_NUM_DYN][9], o[LGX_NUM_DYN][3], S[LGX_NUM_DOF][6], I6[LGX_NUM_DYN][36];
  float H[DN * DN], M[DN * DN];
  float V[LGX_NUM_DYN][6], A[LGX_NUM_DYN][6], F[LGX_NUM_DYN][6];
  float ICroot[4][36], Froot[4][6];          // per leg: composite inertia and force sum at its root
  float Cb[DN], g[DN], Hu[DN], r[DN], u[DN], u2[DN];
  float th[12], thd[12], tgt[12], tex[12], Dimp[12];
  float root[13];
  int impl[12];
  int nc;
};

// per-contact slots in dynamic LDS: [capacity] arrays
struct DenseContacts {
  float (*J)[3 * DN];
  float (*P)[3];
  float (*n)[3];
  float* depth;
  float* mu;
  float (*fs)[3];
  float (*f)[3];
  int* body;
  int* report;
  int* stat;
};

LGX_DEV DenseContacts dense_contacts(float* base, int cap) {
  DenseContacts c;
  c.J = reinterpret_cast<float(*)[3 * DN]>(base);
  c.P = reinterpret_cast<float(*)[3]>(base + cap * 3 * DN);
  c.n = reinterpret_cast<float(*)[3]>(base + cap * (3 * DN + 3));
  c.depth = base + cap * (3 * DN + 6);
  c.mu = base + cap * (3 * DN + 7);
  c.fs = reinterpret_cast<float(*)[3]>(base + cap * (3 * DN + 8));
  c.f = reinterpret_cast<float(*)[3]>(base + cap * (3 * DN + 11));
  int* ib = reinterpret_cast<int*>(base + cap * DCF);
  c.body = ib;
  c.report = ib + cap;
  c.stat = ib + 2 * cap;
  return c;
}

// does dyn body `body`'s chain contain joint `joint` (legs of LD joints)
LGX_DEV bool d_chain_has(int body, int joint, int LD) {
  if (body == 0) return false;
  const int leg = (body - 1) / LD, k = (body - 1) % LD;
  return joint / LD == leg && joint % LD <= k;
}

// column c of body b's 6 x 18 Jacobian (ang; lin at the base origin)
LGX_DEV void d_body_col(const DenseLds& L, int b, int c, int LD, float* col) {
#pragma unroll
  for (int i = 0; i < 6; ++i) col[i] = 0.f;
  if (c < 6) { col[c] = 1.f; return; }
  const int j = c - 6;
  if (d_chain_has(b, j, LD))
#pragma unroll
    for (int i = 0; i < 6; ++i) col[i] = L.S[j][i];
}

LGX_DEV void d_crm(const float* V, const float* s, float* o) {   // V x_m s
  const f3 a = cross(mk3(V[0], V[1], V[2]), mk3(s[0], s[1], s[2]));
  const f3 l = cross(mk3(V[0], V[1], V[2]), mk3(s[3], s[4], s[5])) + cross(mk3(V[3], V[4], V[5]), mk3(s[0], s[1], s[2]));
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = l.x; o[4] = l.y; o[5] = l.z;
}
LGX_DEV void d_crf(const float* V, const float* f, float* o) {   // V x_f f
  const f3 a = cross(mk3(V[0], V[1], V[2]), mk3(f[0], f[1], f[2])) + cross(mk3(V[3], V[4], V[5]), mk3(f[3], f[4], f[5]));
  const f3 l = cross(mk3(V[0], V[1], V[2]), mk3(f[3], f[4], f[5]));
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = l.x; o[4] = l.y; o[5] = l.z;
}

}  // namespace

__global__ void __launch_bounds__(64) lgx_physics_dense_kernel(const lgx_dev_model* __restrict__ DMg,
                                                               const lgx_env_params* __restrict__ P, lgx_buffers B,
                                                               int32_t nsub, int32_t from_actions,
                                                               const float* __restrict__ act_src, int32_t frozen,
                                                               int32_t cap) {
  __shared__ DenseLds L;
  extern __shared__ __attribute__((aligned(16))) float dyn_lds[];
  const DenseContacts Ct = dense_contacts(dyn_lds, cap);
  const lgx_model* __restrict__ M = &DMg->m;
  const int lane = threadIdx.x;
  const int e = blockIdx.x;
  const int N = P->num_envs;
  if (e >= N) return;
  const int LD = M->leg_dof == 6 ? 6 : 3, NL = LGX_NUM_DOF / LD;
  const int ctrl = P->control_type;
  const float dt = M->sim_dt;
  // ---- load: state, clipped actions, position targets (legged_robot.py:85-86, 394-397)
  if (lane < 12) {
    const int j = lane;
    L.th[j] = B.dof_state[(int64_t)e * 24 + 2 * j];
    L.thd[j] = B.dof_state[(int64_t)e * 24 + 2 * j + 1];
    float a = 0.f;
    if (from_actions) a = clampf(act_src[(int64_t)e * 12 + j], -P->clip_actions, P->clip_actions);
    if (ctrl == LGX_CTRL_POS_DRIVE)
      L.tgt[j] = from_actions ? clampf(a * P->action_scale + P->default_dof_pos[j], P->soft_lower[j], P->soft_upper[j])
                              : B.dof_targets[(int64_t)e * 12 + j];
    if (from_actions) {
      B.actions[(int64_t)e * 12 + j] = a;
      if (ctrl == LGX_CTRL_POS_DRIVE) B.dof_targets[(int64_t)e * 12 + j] = L.tgt[j];
    }
  }
  if (lane < 13) L.root[lane] = B.root_states[(int64_t)e * 13 + lane];
  if (frozen) return;
  const float mu_env = B.friction ? B.friction[e] : 1.f;
  const float kn = M->contact_k, cn = M->contact_c, ct = M->friction_c;
  __syncthreads();

  for (int s = 0; s < nsub; ++s) {
    // ---- explicit torques (_compute_torques, legged_robot.py:370-392): caller-provided or P / V / T
    if (lane < 12 && ctrl != LGX_CTRL_POS_DRIVE) {
      const int j = lane;
      float t;
      if (!from_actions) t = B.torques[(int64_t)e * 12 + j];
      else {
        const float a = B.actions[(int64_t)e * 12 + j] * P->action_scale;
        if (ctrl == LGX_CTRL_P) t = P->p_gains[j] * (a + P->default_dof_pos[j] - L.th[j]) - P->d_gains[j] * L.thd[j];
        else if (ctrl == LGX_CTRL_V)
          t = P->p_gains[j] * (a - L.thd[j]) - P->d_gains[j] * (L.thd[j] - B.last_dof_vel[(int64_t)e * 12 + j]) / dt;
        else t = a;
        t = clampf(t, -P->torque_limits[j], P->torque_limits[j]);
      }
      L.tex[j] = t;
    }
    if (lane < 6) L.u[lane] = lane < 3 ? L.root[10 + lane] : L.root[7 + lane - 3];
    else if (lane < DN) L.u[lane] = L.thd[lane - 6];
    for (int q = lane; q < DN * DN; q += 64) L.H[q] = 0.f;
    // ---- one lane per leg chain: kinematics + RNEA velocities / accelerations (A_0 = (0, -w x v - g))
    const m33 R0 = quat_to_mat(L.root[3], L.root[4], L.root[5], L.root[6]);
    const float ub[6] = {L.root[10], L.root[11], L.root[12], L.root[7], L.root[8], L.root[9]};
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 9; ++i) L.R[0][i] = R0.a[i];
      L.o[0][0] = L.o[0][1] = L.o[0][2] = 0.f;
      const f3 wxv = cross(mk3(ub[0], ub[1], ub[2]), mk3(ub[3], ub[4], ub[5]));
#pragma unroll
      for (int i = 0; i < 6; ++i) L.V[0][i] = ub[i];
      L.A[0][0] = L.A[0][1] = L.A[0][2] = 0.f;
      L.A[0][3] = -wxv.x - M->gravity[0]; L.A[0][4] = -wxv.y - M->gravity[1]; L.A[0][5] = -wxv.z - M->gravity[2];
    }
    if (lane < NL) {
      m33 Rp = R0;
      f3 op = mk3(0.f, 0.f, 0.f);
      float Vp[6], Ap[6];
      const f3 wxv = cross(mk3(ub[0], ub[1], ub[2]), mk3(ub[3], ub[4], ub[5]));
#pragma unroll
      for (int i = 0; i < 6; ++i) Vp[i] = ub[i];
      Ap[0] = Ap[1] = Ap[2] = 0.f;
      Ap[3] = -wxv.x - M->gravity[0]; Ap[4] = -wxv.y - M->gravity[1]; Ap[5] = -wxv.z - M->gravity[2];
      for (int k = 0; k < LD; ++k) {
        const int j = LD * lane + k, b = 1 + j;
        m33 Jr;
#pragma unroll
        for (int i = 0; i < 9; ++i) Jr.a[i] = M->joint_rot[j][i];
        const m33 Rjf = mul(Rp, Jr);
        const f3 ob = op + mul(Rp, mk3(M->joint_pos[j][0], M->joint_pos[j][1], M->joint_pos[j][2]));
        const f3 ax = mk3(M->joint_axis[j][0], M->joint_axis[j][1], M->joint_axis[j][2]);
        const f3 aw = mul(Rjf, ax);
        const m33 Rb = mul(Rjf, axis_angle(ax, L.th[j]));
        const f3 ow = cross(ob, aw);
        const float Sj[6] = {aw.x, aw.y, aw.z, ow.x, ow.y, ow.z};
        const float qd = L.thd[j];
        float c6[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) Vp[i] = Vp[i] + Sj[i] * qd;
        d_crm(Vp, Sj, c6);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          Ap[i] = Ap[i] + c6[i] * qd;
          L.S[j][i] = Sj[i];
          L.V[b][i] = Vp[i];
          L.A[b][i] = Ap[i];
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) L.R[b][i] = Rb.a[i];
        L.o[b][0] = ob.x; L.o[b][1] = ob.y; L.o[b][2] = ob.z;
        Rp = Rb;
        op = ob;
      }
    }
    __syncthreads();
    // ---- one lane per body: spatial inertia at the base origin (oracle spatial_inertia) and the
    // body force f_b = I_b A_b + V_b x* I_b V_b
    if (lane < LGX_NUM_DYN) {
      const int b = lane;
      const float* in = M->body_inertia[b];
      const float scale = B.body_mass_scale[(int64_t)e * LGX_NUM_DYN + b];
      m33 R, Ib, RT;
#pragma unroll
      for (int i = 0; i < 9; ++i) R.a[i] = L.R[b][i];
      Ib.a[0] = in[0]; Ib.a[1] = in[3]; Ib.a[2] = in[4]; Ib.a[3] = in[3]; Ib.a[4] = in[1]; Ib.a[5] = in[5];
      Ib.a[6] = in[4]; Ib.a[7] = in[5]; Ib.a[8] = in[2];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) RT.a[3 * i + j] = R.a[3 * j + i];
      m33 Iw = mul(mul(R, Ib), RT);
      const f3 c = mul(R, mk3(M->body_com[b][0], M->body_com[b][1], M->body_com[b][2])) +
                   mk3(L.o[b][0], L.o[b][1], L.o[b][2]);
      const float mass = M->body_mass[b] * scale;
#pragma unroll
      for (int i = 0; i < 9; ++i) Iw.a[i] *= scale;
      const float cc = dot(c, c);
      const float cv[3] = {c.x, c.y, c.z};
      const float sk[9] = {0.f, -c.z, c.y, c.z, 0.f, -c.x, -c.y, c.x, 0.f};
      float I6[36];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          I6[i * 6 + j] = Iw.a[3 * i + j] + mass * ((i == j ? cc : 0.f) - cv[i] * cv[j]);
          I6[(3 + i) * 6 + 3 + j] = i == j ? mass : 0.f;
          I6[i * 6 + 3 + j] = mass * sk[3 * i + j];
          I6[(3 + i) * 6 + j] = mass * sk[3 * j + i];
        }
      float Vb[6], Ab[6], IA[6], IV[6], vf[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) { Vb[i] = L.V[b][i]; Ab[i] = L.A[b][i]; }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        float x = 0.f, y = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j) { x += I6[i * 6 + j] * Ab[j]; y += I6[i * 6 + j] * Vb[j]; }
        IA[i] = x; IV[i] = y;
      }
      d_crf(Vb, IV, vf);
#pragma unroll
      for (int i = 0; i < 6; ++i) L.F[b][i] = IA[i] + vf[i];
#pragma unroll
      for (int i = 0; i < 36; ++i) L.I6[b][i] = I6[i];
    }
    __syncthreads();
    // ---- one lane per leg: composite inertias and subtree forces from the tip (CRBA / RNEA):
    // H[j][k] = S_j . IC_k S_k (k deeper on the chain), H[base][k] = IC_k S_k, C_j = S_j . F_k
    if (lane < NL) {
      const int leg = lane;
      float IC[36], Fs[6];
#pragma unroll
      for (int i = 0; i < 36; ++i) IC[i] = 0.f;
#pragma unroll
      for (int i = 0; i < 6; ++i) Fs[i] = 0.f;
      for (int k = LD - 1; k >= 0; --k) {
        const int j = LD * leg + k, b = 1 + j;
#pragma unroll
        for (int i = 0; i < 36; ++i) IC[i] += L.I6[b][i];
#pragma unroll
        for (int i = 0; i < 6; ++i) Fs[i] += L.F[b][i];
        float Sk[6], Fc[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) Sk[i] = L.S[j][i];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          float x = 0.f;
#pragma unroll
          for (int m = 0; m < 6; ++m) x += IC[i * 6 + m] * Sk[m];
          Fc[i] = x;
        }
        float cj = 0.f;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          L.H[i * DN + 6 + j] = Fc[i];       // base rows / column j (symmetric)
          L.H[(6 + j) * DN + i] = Fc[i];
          cj += Sk[i] * Fs[i];
        }
        L.Cb[6 + j] = cj;
        for (int kk = 0; kk <= k; ++kk) {    // joints j' on the chain from the root down to j
          const int jj = LD * leg + kk;
          float h = 0.f;
#pragma unroll
          for (int i = 0; i < 6; ++i) h += L.S[jj][i] * Fc[i];
          L.H[(6 + jj) * DN + 6 + j] = h;
          L.H[(6 + j) * DN + 6 + jj] = h;
        }
      }
#pragma unroll
      for (int i = 0; i < 36; ++i) L.ICroot[leg][i] = IC[i];
#pragma unroll
      for (int i = 0; i < 6; ++i) L.Froot[leg][i] = Fs[i];
    }
    // ---- drives (implicit PD while within the effort limit) and hard-limit springs
    if (lane >= 32 && lane < 44) {
      const int j = lane - 32;
      float gj = 0.f, dimp = 0.f;
      int impl = 0;
      const float eff = M->dof_effort[j];
      const float th = L.th[j], thd = L.thd[j];
      if (ctrl == LGX_CTRL_POS_DRIVE) {
        const float te = M->kp[j] * (L.tgt[j] - th) - M->kd[j] * thd;
        if (fabsf(te) <= eff) {
          impl = 1;
          dimp += dt * (M->kd[j] + dt * M->kp[j]);
          gj += M->kp[j] * (L.tgt[j] - th);
        } else {
          gj += te > 0.f ? eff : -eff;
        }
      } else {
        gj += L.tex[j];
      }
      if (M->dof_lower[j] < M->dof_upper[j]) {
        if (th < M->dof_lower[j]) {
          dimp += dt * (M->limit_c + dt * M->limit_k);
          gj += M->limit_k * (M->dof_lower[j] - th);
        } else if (th > M->dof_upper[j]) {
          dimp += dt * (M->limit_c + dt * M->limit_k);
          gj -= M->limit_k * (th - M->dof_upper[j]);
        }
      }
      L.g[6 + j] = gj;
      L.Dimp[j] = dimp;
      L.impl[j] = impl;
    } else if (lane >= 44 && lane < 50) {
      L.g[lane - 44] = 0.f;
    }
    if (lane == 63) L.nc = 0;
    __syncthreads();
    // base block and base bias: the base body plus every leg's composite at its root
    if (lane < 36) {
      float h = L.I6[0][lane];
      for (int leg = 0; leg < NL; ++leg) h += L.ICroot[leg][lane];
      L.H[(lane / 6) * DN + lane % 6] = h;
    } else if (lane < 42) {
      const int i = lane - 36;
      float c = L.F[0][i];
      for (int leg = 0; leg < NL; ++leg) c += L.Froot[leg][i];
      L.Cb[i] = c;
    }
    // (H's base block and Cb are read by other lanes below, also when no candidate loop runs)
    __syncthreads();
    // ---- contact candidates: one lane per point, compacted in point order
    const int npts = M->num_points;
    for (int i0 = 0; i0 < npts; i0 += 64) {
      const int i = i0 + lane;
      bool hit = false;
      f3 Pc, n;
      float depth = 0.f;
      int b = 0;
      if (i < npts) {
        b = M->point_dyn[i];
        m33 R;
#pragma unroll
        for (int k = 0; k < 9; ++k) R.a[k] = L.R[b][k];
        const f3 Pp = mul(R, mk3(M->point_pos[i][0], M->point_pos[i][1], M->point_pos[i][2])) +
                      mk3(L.o[b][0], L.o[b][1], L.o[b][2]);
        const float rad = M->point_radius[i];
        depth = ground_contact(P, B, Pp + mk3(L.root[0], L.root[1], L.root[2]), rad, &n, nullptr, 0, 0);
        hit = depth > 0.f;
        Pc = Pp - rad * n;
      }
      const uint64_t mask = __ballot(hit);
      const int base = L.nc;
      if (hit) {
        const int slot = base + __popcll(mask & ((1ull << lane) - 1ull));
        Ct.body[slot] = b;
        Ct.report[slot] = M->point_report[i];
        Ct.P[slot][0] = Pc.x; Ct.P[slot][1] = Pc.y; Ct.P[slot][2] = Pc.z;
        Ct.n[slot][0] = n.x; Ct.n[slot][1] = n.y; Ct.n[slot][2] = n.z;
        Ct.depth[slot] = depth;
        Ct.mu[slot] = 0.5f * (mu_env + M->ground_friction);
        Ct.stat[slot] = 1;
      }
      __syncthreads();
      if (lane == 0) L.nc = base + __popcll(mask);
      __syncthreads();
    }
    const int nc = L.nc;
    // contact point Jacobians (3 x 18): v_P = v_lin + w x P, one lane per (contact, column)
    for (int q = lane; q < nc * DN; q += 64) {
      const int i = q / DN, c = q % DN;
      float col[6];
      d_body_col(L, Ct.body[i], c, LD, col);
      const f3 wxp = cross(mk3(col[0], col[1], col[2]), mk3(Ct.P[i][0], Ct.P[i][1], Ct.P[i][2]));
      Ct.J[i][c] = col[3] + wxp.x;
      Ct.J[i][DN + c] = col[4] + wxp.y;
      Ct.J[i][2 * DN + c] = col[5] + wxp.z;
    }
    // H u
    if (lane >= 32 && lane < 32 + DN) {
      const int c = lane - 32;
      float hu = 0.f;
      for (int k = 0; k < DN; ++k) hu += L.H[c * DN + k] * L.u[k];
      L.Hu[c] = hu;
    }
    __syncthreads();
    // ---- two passes: all penetrating points sticking, then sliding points as Coulomb forces
    for (int pass = 0; pass < 2; ++pass) {
      for (int q = lane; q < DN * DN; q += 64) {     // lower triangle + diagonal of M
        const int a = q / DN, c = q % DN;
        if (c > a) continue;
        float m = L.H[q];
        if (a == c && a >= 6) m += L.Dimp[a - 6];
        for (int i = 0; i < nc; ++i) {
          if (Ct.stat[i] == 0) continue;
          const float wt = (pass == 0 || Ct.stat[i] == 1) ? dt * ct : 0.f;
          const float wn = dt * (cn + dt * kn);
          const float* J = Ct.J[i];
          const float nv[3] = {Ct.n[i][0], Ct.n[i][1], Ct.n[i][2]};
          const float jc[3] = {J[c], J[DN + c], J[2 * DN + c]};
          const float ndc = (wn - wt) * (nv[0] * jc[0] + nv[1] * jc[1] + nv[2] * jc[2]);
          m += J[a] * (wt * jc[0] + ndc * nv[0]) + J[DN + a] * (wt * jc[1] + ndc * nv[1]) +
               J[2 * DN + a] * (wt * jc[2] + ndc * nv[2]);
        }
        L.M[q] = m;
      }
      if (lane >= 32 && lane < 32 + DN) {
        const int a = lane - 32;
        float rv = L.Hu[a] + dt * (L.g[a] - L.Cb[a]);
        for (int i = 0; i < nc; ++i) {
          if (Ct.stat[i] == 0) continue;
          const float* J = Ct.J[i];
          const float jn = J[a] * Ct.n[i][0] + J[DN + a] * Ct.n[i][1] + J[2 * DN + a] * Ct.n[i][2];
          rv += dt * kn * Ct.depth[i] * jn;
          if (pass == 1 && Ct.stat[i] == 2)
            rv += dt * (J[a] * Ct.fs[i][0] + J[DN + a] * Ct.fs[i][1] + J[2 * DN + a] * Ct.fs[i][2]);
        }
        L.r[a] = rv;
      }
      __syncthreads();
      // Cholesky (lower), one lane per row of each column
      for (int j = 0; j < DN; ++j) {
        float sjj = L.M[j * DN + j];
        for (int k = 0; k < j; ++k) sjj -= L.M[j * DN + k] * L.M[j * DN + k];
        const float d = sqrtf(sjj > 1e-20f ? sjj : 1e-20f);
        const int i = lane;
        float t = 0.f;
        if (i > j && i < DN) {
          t = L.M[i * DN + j];
          for (int k = 0; k < j; ++k) t -= L.M[i * DN + k] * L.M[j * DN + k];
        }
        __syncthreads();
        if (lane == j) L.M[j * DN + j] = d;
        if (i > j && i < DN) L.M[i * DN + j] = t / d;
        __syncthreads();
      }
      // substitutions: the solution entries in LDS, one lane per row updating after each pivot
      for (int i = 0; i < DN; ++i) {
        if (lane == 0) L.u2[i] = L.r[i] / L.M[i * DN + i];
        __syncthreads();
        if (lane > i && lane < DN) L.r[lane] -= L.M[lane * DN + i] * L.u2[i];
        __syncthreads();
      }
      for (int i = DN - 1; i >= 0; --i) {
        if (lane == 0) L.u2[i] = L.u2[i] / L.M[i * DN + i];
        __syncthreads();
        if (lane < i) L.u2[lane] -= L.M[i * DN + lane] * L.u2[i];
        __syncthreads();
      }
      if (pass == 0) {   // classify: separating, sliding (Coulomb cone), sticking
        for (int i = lane; i < nc; i += 64) {
          const float* J = Ct.J[i];
          float vp[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            float sv = 0.f;
            for (int a = 0; a < DN; ++a) sv += J[k * DN + a] * L.u2[a];
            vp[k] = sv;
          }
          const f3 nn = mk3(Ct.n[i][0], Ct.n[i][1], Ct.n[i][2]);
          const float vn = vp[0] * nn.x + vp[1] * nn.y + vp[2] * nn.z;
          const float fn = kn * Ct.depth[i] - (cn + dt * kn) * vn;
          const float vt[3] = {vp[0] - vn * nn.x, vp[1] - vn * nn.y, vp[2] - vn * nn.z};
          const float vtn = sqrtf(vt[0] * vt[0] + vt[1] * vt[1] + vt[2] * vt[2]);
          if (fn <= 0.f) Ct.stat[i] = 0;
          else if (ct * vtn > Ct.mu[i] * fn) {
            Ct.stat[i] = 2;
            const float sc = -Ct.mu[i] * fn / vtn;
            Ct.fs[i][0] = sc * vt[0]; Ct.fs[i][1] = sc * vt[1]; Ct.fs[i][2] = sc * vt[2];
          } else Ct.stat[i] = 1;
        }
        __syncthreads();
      }
    }
    // ---- reported contact forces (net force per reporting body, the last substep's)
    if (s == nsub - 1) {
      for (int i = lane; i < nc; i += 64) {
        float f[3] = {0.f, 0.f, 0.f};
        if (Ct.stat[i] != 0) {
          const float* J = Ct.J[i];
          float vp[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            float sv = 0.f;
            for (int a = 0; a < DN; ++a) sv += J[k * DN + a] * L.u2[a];
            vp[k] = sv;
          }
          const float vn = vp[0] * Ct.n[i][0] + vp[1] * Ct.n[i][1] + vp[2] * Ct.n[i][2];
          float fn = kn * Ct.depth[i] - (cn + dt * kn) * vn;
          if (fn < 0.f) fn = 0.f;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const float ft = Ct.stat[i] == 1 ? -ct * (vp[k] - vn * Ct.n[i][k]) : Ct.fs[i][k];
            f[k] = fn * Ct.n[i][k] + ft;
          }
        }
        Ct.f[i][0] = f[0]; Ct.f[i][1] = f[1]; Ct.f[i][2] = f[2];
      }
      __syncthreads();
      if (lane < LGX_MAX_BODIES) {
        float f[3] = {0.f, 0.f, 0.f};
        for (int i = 0; i < nc; ++i)
          if (Ct.report[i] == lane) { f[0] += Ct.f[i][0]; f[1] += Ct.f[i][1]; f[2] += Ct.f[i][2]; }
        float* cfo = B.contact_forces + ((int64_t)e * LGX_MAX_BODIES + lane) * 3;
        cfo[0] = f[0]; cfo[1] = f[1]; cfo[2] = f[2];
      }
    }
    // ---- joint outputs and the root (semi-implicit Euler, quaternion renormalised)
    if (lane < 12) {
      const int j = lane;
      float qd = L.u2[6 + j];
      const float vl = M->dof_vel_limit[j];
      if (vl > 0.f) qd = clampf(qd, -vl, vl);
      if (ctrl == LGX_CTRL_POS_DRIVE && s == nsub - 1) {
        const float eff = M->dof_effort[j];
        float t;
        if (L.impl[j]) t = M->kp[j] * (L.tgt[j] - L.th[j] - dt * L.u2[6 + j]) - M->kd[j] * L.u2[6 + j];
        else t = M->kp[j] * (L.tgt[j] - L.th[j]) - M->kd[j] * L.thd[j];
        B.torques[(int64_t)e * 12 + j] = clampf(t, -eff, eff);
      }
      L.th[j] = L.th[j] + dt * qd;
      L.thd[j] = qd;
    } else if (lane == 32) {
      const f3 w = mk3(L.u2[0], L.u2[1], L.u2[2]), v = mk3(L.u2[3], L.u2[4], L.u2[5]);
      L.root[0] += dt * v.x; L.root[1] += dt * v.y; L.root[2] += dt * v.z;
      const f3 q = mk3(L.root[3], L.root[4], L.root[5]);
      const float qw = L.root[6];
      const f3 wq = cross(w, q);
      float dq[4] = {0.5f * (qw * w.x + wq.x), 0.5f * (qw * w.y + wq.y), 0.5f * (qw * w.z + wq.z), -0.5f * dot(w, q)};
      float qq[4] = {q.x + dt * dq[0], q.y + dt * dq[1], q.z + dt * dq[2], qw + dt * dq[3]};
      const float qn = 1.0f / sqrtf(qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2] + qq[3] * qq[3]);
      L.root[3] = qq[0] * qn; L.root[4] = qq[1] * qn; L.root[5] = qq[2] * qn; L.root[6] = qq[3] * qn;
      L.root[7] = v.x; L.root[8] = v.y; L.root[9] = v.z;
      L.root[10] = w.x; L.root[11] = w.y; L.root[12] = w.z;
    }
    __syncthreads();
  }
  // ---- write back
  if (lane < 12) {
    B.dof_state[(int64_t)e * 24 + 2 * lane] = L.th[lane];
    B.dof_state[(int64_t)e * 24 + 2 * lane + 1] = L.thd[lane];
    if (ctrl != LGX_CTRL_POS_DRIVE && nsub > 0) B.torques[(int64_t)e * 12 + lane] = L.tex[lane];
  }
  if (lane < 13) B.root_states[(int64_t)e * 13 + lane] = L.root[lane];
}

// dynamic LDS bytes of the dense kernel's contact slots for `num_points` candidates
static int lgx_physics_dense_lds(int32_t num_points) { return num_points * (DCF + 3) * 4; }

int lgx_launch_physics_dense(const lgx_dev_model* dm, const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs,
                             int32_t nsub, int32_t from_actions, const float* act_src, hipStream_t stream,
                             int32_t frozen, int32_t num_points) {
  if (!act_src) act_src = b.actions;
  const int cap = num_points > 0 ? num_points : 1;
  LGX_LAUNCH(lgx_physics_dense_kernel, dim3(n_envs), dim3(64), lgx_physics_dense_lds(cap), stream, dm, dp, b, nsub,
             from_actions, act_src, frozen, cap);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

#ifdef LGX_PHASE_CLOCK_BUF
// instrumented builds only (tools/phase_clock.sh): the per-workgroup clock table of the last physics launch
extern "C" int lgx_debug_clock(unsigned long long* out, int32_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lgx_clk_buf), (size_t)min(nblocks, LGX_CLK_MAXB) * 14 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
