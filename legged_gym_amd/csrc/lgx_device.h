// Device helpers shared by the lgx HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lgx.h"

#define LGX_DEV __device__ __forceinline__

// Phase timing of one wave (block 0, thread 0) for kernel tuning: build with
// EXTRA=-DLGX_PHASE_CLOCK (tools/phase_clock.sh); compiled out of the product library.
#ifdef LGX_PHASE_CLOCK
#include <stdio.h>
#define LGX_CLK_DECL(n) LGX_CLK_START uint64_t lgx_clk_acc[n] = {}; uint64_t lgx_clk_t = clock64();
#define LGX_CLK(i) do { const uint64_t _t = clock64(); lgx_clk_acc[i] += _t - lgx_clk_t; lgx_clk_t = _t; } while (0)
#ifdef LGX_PHASE_CLOCK_ALL   // every workgroup's thread 0 (load-balance studies)
#define LGX_CLK_WHO (threadIdx.x == 0)
#else
#define LGX_CLK_WHO (blockIdx.x == 0 && threadIdx.x == 0)
#endif
#ifdef LGX_PHASE_CLOCK_BUF   // per-workgroup record of the last launch in a device table (no printf):
                             // [start, end] (s_memrealtime, 100 MHz) + the phase sums; read by
                             // lgx_debug_clock (lgx_physics.hip)
#define LGX_CLK_MAXB 4096
static __device__ unsigned long long lgx_clk_buf[LGX_CLK_MAXB][14];
#define LGX_CLK_START const unsigned long long lgx_clk_t0 = __builtin_amdgcn_s_memrealtime();
#define LGX_CLK_PRINT(name, n)                                                                        \
  if (threadIdx.x == 0 && blockIdx.x < LGX_CLK_MAXB) {                                                \
    lgx_clk_buf[blockIdx.x][0] = lgx_clk_t0;                                                          \
    lgx_clk_buf[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();                                    \
    for (int _i = 0; _i < n && _i < 12; ++_i) lgx_clk_buf[blockIdx.x][2 + _i] = lgx_clk_acc[_i];      \
  }
#else
#define LGX_CLK_START
#define LGX_CLK_PRINT(name, n)                                                                        \
  if (LGX_CLK_WHO) {   /* one printf per line (lines of concurrent workgroups do not interleave) */   \
    unsigned long long _v[12] = {};                                                                   \
    for (int _i = 0; _i < n && _i < 12; ++_i) _v[_i] = lgx_clk_acc[_i];                               \
    printf("%s cycles: b=%d 0=%llu 1=%llu 2=%llu 3=%llu 4=%llu 5=%llu 6=%llu 7=%llu 8=%llu 9=%llu "   \
           "10=%llu 11=%llu\n", name, (int)blockIdx.x, _v[0], _v[1], _v[2], _v[3], _v[4], _v[5], _v[6],  \
           _v[7], _v[8], _v[9], _v[10], _v[11]);                                                       \
  }
#endif
#else
#define LGX_CLK_DECL(n)
#define LGX_CLK(i) do { } while (0)
#define LGX_CLK_PRINT(name, n)
#endif

// ---------------------------------------------------------------- Philox4x32-10 uniforms
// Same stream as the oracle's lgxo_uniform: counter (env, slot/4, step, tag), key = seed.
// Philox-4x32-10 block of draw slots (4q .. 4q+3): one counter per 4 consecutive slots
LGX_DEV void lgx_uniform4(uint64_t seed, int32_t env, int32_t slot4, int64_t step, uint32_t tag, float out[4]) {
  uint32_t c0 = (uint32_t)env, c1 = (uint32_t)slot4, c2 = (uint32_t)step;
  uint32_t c3 = tag ^ ((uint32_t)((uint64_t)step >> 32) << 8);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  const float s = 1.0f / 16777216.0f;
  out[0] = (float)(c0 >> 8) * s; out[1] = (float)(c1 >> 8) * s;
  out[2] = (float)(c2 >> 8) * s; out[3] = (float)(c3 >> 8) * s;
}

LGX_DEV float lgx_uniform(uint64_t seed, int32_t env, int32_t slot, int64_t step, uint32_t tag) {
  float u[4];
  lgx_uniform4(seed, env, slot >> 2, step, tag, u);
  return (slot & 3) == 0 ? u[0] : (slot & 3) == 1 ? u[1] : (slot & 3) == 2 ? u[2] : u[3];
}

// ---------------------------------------------------------------- small vector math
struct f3 { float x, y, z; };
LGX_DEV f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
LGX_DEV f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
LGX_DEV f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
LGX_DEV f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
LGX_DEV float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
LGX_DEV f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

struct m33 { float a[9]; };
LGX_DEV f3 mul(const m33& R, f3 v) {
  return f3{R.a[0] * v.x + R.a[1] * v.y + R.a[2] * v.z, R.a[3] * v.x + R.a[4] * v.y + R.a[5] * v.z,
            R.a[6] * v.x + R.a[7] * v.y + R.a[8] * v.z};
}
LGX_DEV m33 mul(const m33& A, const m33& B) {
  m33 C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C.a[3 * i + j] = A.a[3 * i] * B.a[j] + A.a[3 * i + 1] * B.a[3 + j] + A.a[3 * i + 2] * B.a[6 + j];
  return C;
}
LGX_DEV m33 quat_to_mat(float x, float y, float z, float w) {
  m33 R;
  R.a[0] = 1 - 2 * (y * y + z * z); R.a[1] = 2 * (x * y - z * w);     R.a[2] = 2 * (x * z + y * w);
  R.a[3] = 2 * (x * y + z * w);     R.a[4] = 1 - 2 * (x * x + z * z); R.a[5] = 2 * (y * z - x * w);
  R.a[6] = 2 * (x * z - y * w);     R.a[7] = 2 * (y * z + x * w);     R.a[8] = 1 - 2 * (x * x + y * y);
  return R;
}
LGX_DEV m33 axis_angle(f3 a, float th) {
  float s, c;
  sincosf(th, &s, &c);
  float t = 1 - c;
  m33 R;
  R.a[0] = t * a.x * a.x + c;       R.a[1] = t * a.x * a.y - s * a.z; R.a[2] = t * a.x * a.z + s * a.y;
  R.a[3] = t * a.x * a.y + s * a.z; R.a[4] = t * a.y * a.y + c;       R.a[5] = t * a.y * a.z - s * a.x;
  R.a[6] = t * a.x * a.z - s * a.y; R.a[7] = t * a.y * a.z + s * a.x; R.a[8] = t * a.z * a.z + c;
  return R;
}

// isaacgym.torch_utils semantics, xyzw
LGX_DEV f3 quat_rotate_inverse(float qx, float qy, float qz, float qw, f3 v) {
  f3 q = mk3(qx, qy, qz);
  float a = 2.0f * qw * qw - 1.0f;
  f3 c = cross(q, v);
  float d = dot(q, v);
  return f3{v.x * a - c.x * qw * 2.0f + q.x * d * 2.0f, v.y * a - c.y * qw * 2.0f + q.y * d * 2.0f,
            v.z * a - c.z * qw * 2.0f + q.z * d * 2.0f};
}
LGX_DEV f3 quat_apply(float qx, float qy, float qz, float qw, f3 v) {
  f3 q = mk3(qx, qy, qz);
  f3 t = 2.0f * cross(q, v);
  f3 u = cross(q, t);
  return f3{v.x + qw * t.x + u.x, v.y + qw * t.y + u.y, v.z + qw * t.z + u.z};
}

LGX_DEV float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// quad (4-lane) all-reduce: lanes 4e..4e+3 own one env
// Cross-lane moves on the DPP path (a VALU modifier) instead of ds_bpermute (the LDS crossbar):
// dpp_mov<CTRL> returns the value of the lane selected by the DPP control word.
template <int CTRL>
LGX_DEV float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                              CTRL, 0xF, 0xF, false));
}
LGX_DEV float lane_xor1(float v) { return dpp_mov<0xB1>(v); }   // quad_perm [1,0,3,2]
LGX_DEV float lane_xor2(float v) { return dpp_mov<0x4E>(v); }   // quad_perm [2,3,0,1]
// xor 4 / xor 8 inside a 16-lane row: row_shl:n (from lane + n) or row_shr:n (from lane - n)
LGX_DEV float lane_xor4(float v) {
  const float up = dpp_mov<0x104>(v), dn = dpp_mov<0x114>(v);
  return (threadIdx.x & 4) ? dn : up;
}
LGX_DEV float lane_xor8(float v) {
  const float up = dpp_mov<0x108>(v), dn = dpp_mov<0x118>(v);
  return (threadIdx.x & 8) ? dn : up;
}

// DPP source operand meant to fold into the consuming VALU op (bound_ctrl with full masks: the
// compiler's DPP combine turns `v + dpp_src(v)` into one v_add_f32_dpp)
template <int CTRL>
LGX_DEV float dpp_src(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// sum over the 4 lanes of a quad; every lane gets the bitwise-identical ((a+b)+(c+d)) value
// (float addition is commutative)
LGX_DEV float quad_sum(float v) {
  v += dpp_src<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_src<0x4E>(v);   // quad_perm [2,3,0,1]
  return v;
}

// sum over the 4 quads of a 16-lane row (lanes r, r^4, r^8, r^12) in lane_xor4 / lane_xor8's order
// ((v_p + v_p^1) + (v_p^2 + v_p^3)) for quad index p, on DPP adds: row_ror:4 brings quad p-1, row_ror:12
// quad p+1 - the partner p^1 for odd / even p - then row_ror:8 brings p^2.  Every lane of the row gets
// the same value (float addition is commutative), and the same as the shuffle form.
LGX_DEV float row_quads_sum(float v) {
  const float b = v + dpp_src<0x124>(v);   // row_ror:4  : v_p + v_(p-1)
  const float c = v + dpp_src<0x12C>(v);   // row_ror:12 : v_p + v_(p+1)
  const float a = (threadIdx.x & 4) ? b : c;
  return a + dpp_src<0x128>(a);            // row_ror:8  : + a_(p^2)
}

// triangulated heightfield (diagonal (i,j)-(i+1,j+1), isaacgym terrain_utils trimesh).
// Optional LDS patch: samples (i, j) with 0 <= i - pi0, j - pj0 < LGX_HF_PATCH are read from
// `patch` (a copy of the same int16 samples), others from H: identical values either way.
#ifndef LGX_HF_PATCH
#define LGX_HF_PATCH 16
#endif
LGX_DEV float ground_height(const lgx_env_params* __restrict__ P, const int16_t* __restrict__ H, int rows, int cols,
                            float x, float y, f3* n, const int16_t* patch = nullptr, int pi0 = 0, int pj0 = 0) {
  if (P->terrain_kind == 0 || H == nullptr) { *n = mk3(0.f, 0.f, 1.f); return 0.0f; }
  float hs = P->horizontal_scale, vs = P->vertical_scale;
  float u = (x + P->border_size) / hs, v = (y + P->border_size) / hs;
  int i = (int)floorf(u), j = (int)floorf(v);
  i = min(max(i, 0), rows - 2);
  j = min(max(j, 0), cols - 2);
  float fu = clampf(u - (float)i, 0.f, 1.f), fv = clampf(v - (float)j, 0.f, 1.f);
  float h00, h10, h01, h11;
  const int li = i - pi0, lj = j - pj0;
  if (patch && (unsigned)li < LGX_HF_PATCH - 1 && (unsigned)lj < LGX_HF_PATCH - 1) {
    const int16_t* q = patch + li * LGX_HF_PATCH + lj;
    h00 = q[0] * vs; h10 = q[LGX_HF_PATCH] * vs; h01 = q[1] * vs; h11 = q[LGX_HF_PATCH + 1] * vs;
  } else {
    h00 = H[i * cols + j] * vs; h10 = H[(i + 1) * cols + j] * vs;
    h01 = H[i * cols + j + 1] * vs; h11 = H[(i + 1) * cols + j + 1] * vs;
  }
  float gx, gy, h;
  if (fu >= fv) { gx = (h10 - h00) / hs; gy = (h11 - h10) / hs; h = h00 + fu * (h10 - h00) + fv * (h11 - h10); }
  else          { gx = (h11 - h01) / hs; gy = (h01 - h00) / hs; h = h00 + fv * (h01 - h00) + fu * (h11 - h01); }
  float inv = 1.0f / sqrtf(gx * gx + gy * gy + 1.0f);
  *n = mk3(-gx * inv, -gy * inv, inv);
  return h;
}
