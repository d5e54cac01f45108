// Split-bf16 evaluation of the PPO-update GEMM products on the bf16 MFMA
// (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate; gfx950 has no xf32/TF32 path).
//
// Every f32 operand is split, round-to-nearest, into three bf16 limbs
//   x = x0 + x1 + x2 + e,   x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1),
//   |x1| <= 2^-8 |x0|, |x2| <= 2^-8 |x1|, |e| <= 2^-24 |x|   (both subtractions are exact in f32),
// and a*b is evaluated as the six limb products of order <= 2,
//   a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0),
// each product of two bf16 limbs exact in the f32 accumulator.  The dropped terms (a1 b2, a2 b1,
// a2 b2) and the split residues are at the level of one f32 product rounding (2^-24 |a b|; a few
// times that in the worst case, far less on average since the limb ratios are spread over the
// half-ulp range), and each 16-k MFMA rounds the accumulator once per limb product (6 roundings
// per 16 k against 16 for the fmaf chain): the result is f32-accurate (tests/test_gpu_gemm.py:
// max / mean error vs float64 within 1.25x of the exact-f32 MFMA's on the same operands).
// 6 MFMAs at 1/16 the cost of the f32 MFMA's 8 per 16 k: a 2.67x higher arithmetic roof
// (417 TF/s of f32 products against 157 TF/s).
//
// Same argument block, tile order (persistent workgroups, XCD-contiguous tile ranges) and fused
// epilogues as gemm_nt_kernel (lgx_gemm_common.h).  Differences:
//   * LDS rows hold [limb][32 k] bf16: 3 x 64 B + 16 B pad = 208 B, row starts 52 banks apart
//     (conflict-free ds_read_b128 fragment reads in all four 16-lane groups); lane (r, h) of a
//     32x32x16 MFMA reads k = 8h .. 8h+7 of its row (A) / column (B): one ds_read_b128 per limb;
//   * the A operand (activations) is split once per element on its way into LDS
//     (v_cvt_pk_bf16_f32 + exact f32 subtractions); the B operand (weights) comes pre-split from
//     HBM (x3_limb_off layout, lgx_split_bf16 / the Adam step's limb mirrors) and is copied
//     into LDS as 16-byte chunks - splitting B in the kernel would redo it for every one of the
//     M / 128 row tiles;
//   * 106 KB of LDS (two stages): one workgroup of 8 waves per CU; a three-slot software pipeline
//     over the workgroup's (tile, K stage) slots: slot q's MFMAs run while slot q+1's staged data
//     is split / copied into the other LDS buffer and slot q+2's global loads are in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "lgx_gemm_common.h"
#include "lgx_internal.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));

constexpr int NWX = 4;                           // waves per workgroup (2 x 2 waves of 64 x 64)
constexpr int X3_ROW = 3 * BK * 2 + 16;          // bytes per LDS row (3 limbs of 32 bf16 + pad)
constexpr int X3_TILE = BM * X3_ROW;             // one operand tile: 26,624 B
constexpr int X3_LDS = 2 * X3_TILE;              // one stage (A, B): 53,248 B -> 2 workgroups per CU
constexpr int LIMB_ROW = 3 * BK;                 // bf16 per (row, 32-k block) of a pre-split operand
constexpr int BCH = BN * LIMB_ROW * 2 / 16 / (64 * NWX);   // 16-byte B chunks per thread per stage (3)
#ifndef X3_INTERLEAVE
#define X3_INTERLEAVE 1
#endif

__device__ __forceinline__ void split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  lgx_split2(x0, x1, l0, l1, l2);   // (lgx_internal.h)
}

__device__ __forceinline__ void store_split4(char* row, int c, const float4& v) {
  uint32_t a0, a1, a2, b0, b1, b2;
  split2(v.x, v.y, a0, a1, a2);
  split2(v.z, v.w, b0, b1, b2);
  *reinterpret_cast<uint2*>(row + 2 * c) = make_uint2(a0, b0);
  *reinterpret_cast<uint2*>(row + 2 * BK + 2 * c) = make_uint2(a1, b1);
  *reinterpret_cast<uint2*>(row + 4 * BK + 2 * c) = make_uint2(a2, b2);
}

// Register staging of one K stage: A as f32 (split on the way into LDS); B as f32 or, pre-split,
// as 16-byte limb chunks (chunk i of thread t: tile row (t + 512 i) / 12, 16-B column % 12).
template <bool BS>
struct StageX {
  float4 a[Cfg<NWX>::NL];
  typename std::conditional<BS, uint4, float4>::type b[BS ? BCH : Cfg<NWX>::NL];
};
template <bool BS>
struct OffsX {
  uint32_t a[Cfg<NWX>::NL];
  uint32_t b[BS ? BCH : Cfg<NWX>::NL];   // f32 B: element offsets; pre-split B: byte offsets
};

template <bool BS>
__device__ __forceinline__ void offs_x(OffsX<BS>& o, const GemmArgs& g, int64_t m_base, int n_base, int kb, int tid) {
#pragma unroll
  for (int i = 0; i < Cfg<NWX>::NL; ++i) {
    const int row = (tid >> 3) + Cfg<NWX>::RSTEP * i;
    o.a[i] = (uint32_t)(min(m_base + row, g.M - 1) * g.lda);   // rows past M load row M-1 (discarded)
  }
  if (BS) {   // tiled pre-split layout (x3_limb_off): limb cc / 4, 16-byte k-chunk cc % 4 of row n
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int ch = tid + 64 * NWX * i, row = ch / 12, cc = ch - 12 * row;
      o.b[i] = (uint32_t)((n_base / BN) * kb * (BN * LIMB_ROW * 2) + (cc >> 2) * (BN * BK * 2) + row * (BK * 2) +
                          (((cc & 3) ^ ((row >> 2) & 3)) << 4));
    }
  } else {
#pragma unroll
    for (int i = 0; i < Cfg<NWX>::NL; ++i) o.b[i] = (uint32_t)((int64_t)(n_base + (tid >> 3) + Cfg<NWX>::RSTEP * i) * g.ldb);
  }
}

template <bool BS>
__device__ __forceinline__ void load_x(StageX<BS>& st, const GemmArgs& g, int z, const OffsX<BS>& o, int t, int c) {
  const int K = g.K;
  const uint32_t kc = (uint32_t)min(t * BK + c, K - 4);   // branch-free tail: zeroed when stored
  const char* Ab = reinterpret_cast<const char*>(g.A + z * g.sa);
#pragma unroll
  for (int i = 0; i < Cfg<NWX>::NL; ++i) st.a[i] = *reinterpret_cast<const float4*>(Ab + (uint32_t)((o.a[i] + kc) * 4u));
  if constexpr (BS) {
    const int kb = (K + BK - 1) / BK;
    const char* Bb = reinterpret_cast<const char*>(g.Bs) + (int64_t)z * g.N * kb * (LIMB_ROW * 2) + t * (BN * LIMB_ROW * 2);
#pragma unroll
    for (int i = 0; i < BCH; ++i) st.b[i] = *reinterpret_cast<const uint4*>(Bb + o.b[i]);
  } else {
    const char* Bb = reinterpret_cast<const char*>(g.B + z * g.sb);
#pragma unroll
    for (int i = 0; i < Cfg<NWX>::NL; ++i)
      st.b[i] = *reinterpret_cast<const float4*>(Bb + (uint32_t)((o.b[i] + kc) * 4u));
  }
}

template <bool BS>
__device__ __forceinline__ void store_x(const StageX<BS>& st, char* __restrict__ la, char* __restrict__ lb, bool in,
                                        int tid) {
  const int c = (tid & 7) * 4, r0 = tid >> 3;
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < Cfg<NWX>::NL; ++i) store_split4(la + (r0 + Cfg<NWX>::RSTEP * i) * X3_ROW, c, in ? st.a[i] : zero);
  if constexpr (BS) {
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int ch = tid + 64 * NWX * i, row = ch / 12, cc = ch - 12 * row;
      *reinterpret_cast<uint4*>(lb + row * X3_ROW + cc * 16) = st.b[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < Cfg<NWX>::NL; ++i)
      store_split4(lb + (r0 + Cfg<NWX>::RSTEP * i) * X3_ROW, c, in ? st.b[i] : zero);
  }
}

struct X3Frag {
  bf16x8 a[Cfg<NWX>::WI][3], b[Cfg<NWX>::WJ][3];
};

__device__ __forceinline__ void x3_read(X3Frag& f, const char* __restrict__ la, const char* __restrict__ lb, int wm,
                                        int wn, int r, int h, int s) {
  constexpr int WI = Cfg<NWX>::WI, WJ = Cfg<NWX>::WJ;
  const int ko = 2 * (16 * s + 8 * h);
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int l = 0; l < 3; ++l)
      f.a[i][l] = *reinterpret_cast<const bf16x8*>(la + (wm * 32 * WI + 32 * i + r) * X3_ROW + l * 2 * BK + ko);
#pragma unroll
  for (int j = 0; j < WJ; ++j)
#pragma unroll
    for (int l = 0; l < 3; ++l)
      f.b[j][l] = *reinterpret_cast<const bf16x8*>(lb + (wn * 32 * WJ + 32 * j + r) * X3_ROW + l * 2 * BK + ko);
}

// The MFMA takes the B fragment as its row operand and the A fragment as its column operand,
// so the accumulator is C transposed: acc[i][j][e] = C[m0 + 32i + r][n0 + 32j + 8(e >> 2) + 4h +
// (e & 3)] - every lane holds runs of 4 consecutive columns of one row, stored as 16-byte
// vectors by the epilogue (a quarter of the store instructions of the column layout).
__device__ __forceinline__ void x3_mma(const X3Frag& f, Acc<NWX>& acc) {
  // small terms first (they are the ones the accumulator's rounding would otherwise swamp last)
#pragma unroll
  for (int i = 0; i < Cfg<NWX>::WI; ++i)
#pragma unroll
    for (int j = 0; j < Cfg<NWX>::WJ; ++j) {
      f32x16 c = acc[i][j];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][2], f.a[i][0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][1], f.a[i][1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][0], f.a[i][2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][1], f.a[i][0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][0], f.a[i][1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j][0], f.a[i][0], c, 0, 0, 0);
      acc[i][j] = c;
    }
}

__device__ __forceinline__ float4 q4(const f32x16& v, int q) {
  return make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// Epilogue of the transposed accumulator layout: 16-byte row-contiguous loads / stores.  Rows past
// M are neither stored nor summed.  DELU_COLSUM: per-lane column partials over the wave's rows,
// butterfly over the 32 lanes of each half (same columns), then the wave rows in a fixed order
// (bitwise reproducible).
template <int EPI>
__device__ __forceinline__ void epilogue_t(const GemmArgs& g, const Acc<NWX>& acc, const TileId& T, int wm, int wn,
                                           int r, int h, float* red) {
  constexpr int WI = Cfg<NWX>::WI, WJ = Cfg<NWX>::WJ, WGM = Cfg<NWX>::WGM;
  const int64_t m0 = T.mt * BM + wm * 32 * WI;
  const int n0 = T.nt * BN + wn * 32 * WJ;
  const int64_t ldc = g.ldc;
  float* C = g.C + T.z * g.sc + n0 + 4 * h;
  float4 cs[WJ][4];
  if (EPI == LGX_GEMM_DELU_COLSUM) {
    const float* Y = g.Y + T.z * g.sc + n0 + 4 * h;
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) cs[j][q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const bool ok = m0 + 32 * i + r < g.M;
      const int64_t ro = min(m0 + 32 * i + r, g.M - 1) * ldc;   // rows past M read row M-1, store nothing
      float4 y[WJ][4];
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) y[j][q] = *reinterpret_cast<const float4*>(Y + ro + 32 * j + 8 * q);
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 d = q4(acc[i][j], q);
          d.x *= elu_grad_from_out(y[j][q].x);
          d.y *= elu_grad_from_out(y[j][q].y);
          d.z *= elu_grad_from_out(y[j][q].z);
          d.w *= elu_grad_from_out(y[j][q].w);
          if (ok) {
            *reinterpret_cast<float4*>(C + ro + 32 * j + 8 * q) = d;
            cs[j][q].x += d.x;
            cs[j][q].y += d.y;
            cs[j][q].z += d.z;
            cs[j][q].w += d.w;
          }
        }
    }
#pragma unroll
    for (int sh = 1; sh < 32; sh <<= 1)
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          cs[j][q].x += __shfl_xor(cs[j][q].x, sh);
          cs[j][q].y += __shfl_xor(cs[j][q].y, sh);
          cs[j][q].z += __shfl_xor(cs[j][q].z, sh);
          cs[j][q].w += __shfl_xor(cs[j][q].w, sh);
        }
    // red[WGM][BN]: lane (0, h) of each wave writes its 16 x WJ columns
    const int cl = wn * 32 * WJ + 4 * h;
    if (r == 0) {
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(red + wm * BN + cl + 32 * j + 8 * q) = cs[j][q];
    }
    __syncthreads();
    if (wm == 0 && h == 0) {
      float* P = g.partials + T.mt * ((int64_t)g.batch * g.N) + (int64_t)T.z * g.N + T.nt * BN;
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        const int col = wn * 32 * WJ + 32 * j + r;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WGM; ++w) v += red[w * BN + col];   // fixed order
        P[col] = v;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        cs[j][q] = EPI == LGX_GEMM_BIAS_ELU
                       ? *reinterpret_cast<const float4*>(g.bias + (int64_t)T.z * g.N + n0 + 32 * j + 8 * q + 4 * h)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if (m0 + 32 * i + r >= g.M) continue;
      const int64_t ro = (m0 + 32 * i + r) * ldc;
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v = q4(acc[i][j], q);
          if (EPI == LGX_GEMM_BIAS_ELU) {
            v.x = elu_f(v.x + cs[j][q].x);
            v.y = elu_f(v.y + cs[j][q].y);
            v.z = elu_f(v.z + cs[j][q].z);
            v.w = elu_f(v.w + cs[j][q].w);
          }
          *reinterpret_cast<float4*>(C + ro + 32 * j + 8 * q) = v;
        }
    }
  }
}

// Persistent workgroups over XCD-contiguous tile ranges (as gemm_nt_kernel).  Per K stage: barrier
// (LDS free), the staged registers are split / copied into LDS, barrier, the next stage's global
// loads are issued (the next tile's first stage after a tile's last), then the stage's 48 MFMAs
// per wave.  Two workgroups per CU: one's staging, barriers and epilogue run under the other's
// MFMAs.
template <int EPI, bool BS>
__global__ void __launch_bounds__(64 * NWX, 2) gemm_nt_x3_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char x3lds[];   // X3_LDS bytes
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave / Cfg<NWX>::WGN, wn = wave % Cfg<NWX>::WGN;
  const int ntn = g.N / BN;
  const int64_t total = ((g.M + BM - 1) / BM) * ntn * g.batch;
  const int xcd = blockIdx.x & 7;
  const int64_t wg_per_xcd = gridDim.x >> 3;     // grid is a multiple of 8
  const int64_t lo = xcd * total / 8, hi = (xcd + 1) * total / 8;
  int64_t tile = lo + (blockIdx.x >> 3);
  if (tile >= hi) return;
  const int K = g.K;
  const int nst = (K + BK - 1) / BK;
  const int c = (tid & 7) * 4;
  char* la = x3lds;
  char* lb = x3lds + X3_TILE;

  TileId T = decode_tile(tile, ntn, g.batch);
  OffsX<BS> o;
  offs_x<BS>(o, g, T.mt * BM, T.nt * BN, nst, tid);
  StageX<BS> st;
  load_x<BS>(st, g, T.z, o, 0, c);
  for (;;) {
    const int64_t next = tile + wg_per_xcd;
    const bool has_next = next < hi;
    const TileId Tn = decode_tile(has_next ? next : tile, ntn, g.batch);
    Acc<NWX> acc;
#pragma unroll
    for (int i = 0; i < Cfg<NWX>::WI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg<NWX>::WJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int t = 0; t < nst; ++t) {
      __syncthreads();                                     // every wave is done reading the LDS stage
      store_x<BS>(st, la, lb, t * BK + BK <= K || t * BK + c < K, tid);
      __syncthreads();
      if (t + 1 < nst) {
        load_x<BS>(st, g, T.z, o, t + 1, c);
      } else if (has_next) {                               // the next tile's first stage
        offs_x<BS>(o, g, Tn.mt * BM, Tn.nt * BN, nst, tid);
        load_x<BS>(st, g, Tn.z, o, 0, c);
      }
      X3Frag f0, f1;
      x3_read(f0, la, lb, wm, wn, r, h, 0);
      x3_read(f1, la, lb, wm, wn, r, h, 1);
#ifndef X3_NO_MFMA
      x3_mma(f0, acc);
      x3_mma(f1, acc);
#else
      acc[0][0][0] += (float)f0.a[0][0][0] + (float)f1.b[1][2][3];
#endif
    }
#ifndef X3_NO_EPI
    __syncthreads();     // the LDS stage is reused as the column-sum scratch
    epilogue_t<EPI>(g, acc, T, wm, wn, r, h, reinterpret_cast<float*>(x3lds));
#else
    if (acc[0][0][0] == 12345.f) g.C[0] = acc[1][1][3];
#endif
    if (!has_next) break;
    tile = next;
    T = Tn;
  }
}

// ---------------------------------------------------------------------------------------- weights
// Pre-split operand: out[b][n][k] = transpose ? src[b][k][n] : src[b][n][k] as RNE bf16 limbs in
// the layout the kernel copies, dst[b*dst_bs + n*dst_ld + (k/32)*96 + limb*32 + k%32], zero for
// k >= K up to the 32-k block.  One thread per (b, n, k).
struct SplitJobs {
  lgx_copy2d_job job[LGX_MAX_REDUCE_JOBS];
  int64_t start[LGX_MAX_REDUCE_JOBS + 1];
  int32_t njobs;
};

__global__ void __launch_bounds__(256) split_rows_kernel(SplitJobs J) {
  const int64_t gi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gi >= J.start[J.njobs]) return;
  int ji = 0;
  while (ji + 1 < J.njobs && gi >= J.start[ji + 1]) ++ji;
  const lgx_copy2d_job& jb = J.job[ji];
  const int tr = jb.transpose & 1;
  const int nout = tr ? jb.cols : jb.rows, kout = tr ? jb.rows : jb.cols;
  const int kp = (kout + BK - 1) / BK * BK;
  int64_t l = gi - J.start[ji];
  const int k = (int)(l % kp);
  l /= kp;
  const int n = (int)(l % nout);
  const int b = (int)(l / nout);
  float x = 0.f;
  if (k < kout) x = jb.src[b * jb.src_bs + (tr ? (int64_t)k * jb.src_ld + n : (int64_t)n * jb.src_ld + k)];
  uint16_t* d = reinterpret_cast<uint16_t*>(jb.dst) + b * jb.dst_bs + x3_limb_off(n, k, 0, kp / BK);
  uint32_t l0, l1, l2;
  split2(x, 0.f, l0, l1, l2);
  d[0] = (uint16_t)l0;                 // limb l at + l * 128 * 32 (x3_limb_off)
  d[BN * BK] = (uint16_t)l1;
  d[2 * BN * BK] = (uint16_t)l2;
}

}  // namespace

// lgx_gemm_nt's split-bf16 path (lgx_gemm.hip checks the common arguments first): the pipelined
// kernel (lgx_gemm_x3p.hip) whenever B is pre-split and K % 32 == 0, else the register-staged one
int lgx_gemm_nt_split(const lgx_gemm_args& a, int cus, void* stream_) {
  if (a.Bs && a.K % BK == 0) return lgx_gemm_nt_x3p(a, cus, stream_);
  if (a.epi == LGX_GEMM_DELU)
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: LGX_GEMM_DELU needs a pre-split B (Bs) and K % 32 == 0");
  const hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  GemmArgs g{a.M, a.N, a.K, a.batch, a.epi, a.A, a.lda, a.sa, a.B, a.ldb, a.sb, a.C, a.ldc, a.sc, a.bias, a.Y,
             a.partials, 0, a.Bs};
  const int64_t tiles = ((a.M + BM - 1) / BM) * (a.N / BN) * a.batch;
  static const bool attrs = [] {
    bool ok = true;
    const void* ks[] = {reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_PLAIN, false>),
                        reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_BIAS_ELU, false>),
                        reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_DELU_COLSUM, false>),
                        reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_PLAIN, true>),
                        reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_BIAS_ELU, true>),
                        reinterpret_cast<const void*>(&gemm_nt_x3_kernel<LGX_GEMM_DELU_COLSUM, true>)};
    for (const void* k : ks) ok &= hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, X3_LDS) == hipSuccess;
    return ok;
  }();
  if (!attrs) return lgx_fail(LGX_EHIP, "lgx_gemm_nt: hipFuncSetAttribute (dynamic LDS) failed");
  if (a.Bs && (((uintptr_t)a.Bs & 15) || (int64_t)a.N * ((a.K + BK - 1) / BK) * (LIMB_ROW * 2) >= (1ll << 31)))
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: pre-split B must be 16-byte aligned and < 2 GB per batch entry");
  // persistent: 2 workgroups per CU (53 KB of LDS each), a multiple of 8 (XCD tile ranges)
  const int64_t per_xcd = (tiles + 7) / 8;
  const int64_t wgs = 8 * std::min<int64_t>(per_xcd, std::max(1, 2 * cus / 8));
  const dim3 grid((unsigned)wgs), block(64 * NWX);
#define LGX_X3(EPI, BS) LGX_LAUNCH((gemm_nt_x3_kernel<EPI, BS>), grid, block, X3_LDS, stream, g)
  if (a.Bs) {
    if (a.epi == LGX_GEMM_BIAS_ELU) LGX_X3(LGX_GEMM_BIAS_ELU, true);
    else if (a.epi == LGX_GEMM_DELU_COLSUM) LGX_X3(LGX_GEMM_DELU_COLSUM, true);
    else LGX_X3(LGX_GEMM_PLAIN, true);
  } else {
    if (a.epi == LGX_GEMM_BIAS_ELU) LGX_X3(LGX_GEMM_BIAS_ELU, false);
    else if (a.epi == LGX_GEMM_DELU_COLSUM) LGX_X3(LGX_GEMM_DELU_COLSUM, false);
    else LGX_X3(LGX_GEMM_PLAIN, false);
  }
#undef LGX_X3
  return lgx_hip_status("lgx_gemm_nt");
}

extern "C" int64_t lgx_split_bf16_elems(int32_t n, int32_t k) { return (int64_t)n * ((k + BK - 1) / BK) * LIMB_ROW; }

extern "C" int lgx_split_bf16(const lgx_copy2d_job* jobs, int32_t njobs, void* stream) {
  if (!jobs || njobs <= 0 || njobs > LGX_MAX_REDUCE_JOBS) return lgx_fail(LGX_EINVAL, "lgx_split_bf16: bad job count");
  SplitJobs J;
  int64_t total = 0;
  J.njobs = njobs;
  for (int i = 0; i < njobs; ++i) {
    const lgx_copy2d_job& j = jobs[i];
    const int tr = j.transpose & 1;
    const int nout = tr ? j.cols : j.rows, kout = tr ? j.rows : j.cols;
    if (!j.src || !j.dst || j.rows <= 0 || j.cols <= 0 || j.batch <= 0 || j.src_ld < j.cols || nout % BN ||
        j.dst_bs < lgx_split_bf16_elems(nout, kout))
      return lgx_fail(LGX_EINVAL, "lgx_split_bf16: bad job (output rows % 128, dst_bs)");
    J.job[i] = j;
    J.start[i] = total;
    total += (int64_t)j.batch * nout * ((kout + BK - 1) / BK * BK);
  }
  J.start[njobs] = total;
  if (total > (1ll << 31)) return lgx_fail(LGX_EINVAL, "lgx_split_bf16: too large");
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), J);
  return lgx_hip_status("lgx_split_bf16");
}
