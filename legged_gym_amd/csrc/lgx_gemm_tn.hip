// Weight-gradient GEMM of the PPO update (rsl_rl PPO.update backward, legged_robot_config.py:226-239),
// split-K over row slices:
//   C[z][s][n][c] = sum_{m in slice s} A[z][m][n] * B[z][m][c],   slice s = rows [s Ms, (s+1) Ms)
// i.e. dW_k = dZ_k^T Y_{k-1} per network z (actor, critic) and row slice s; lgx_reduce_slices sums
// the slices into the flat gradient.  Replaces the library f32 bmm over slices.
//
// Same f32-accurate arithmetic as the split-bf16 path of lgx_gemm_nt (lgx_gemm_split.hip): both
// operands split into three RNE bf16 limbs, six limb products on v_mfma_f32_32x32x16_bf16.
// Both operands are row-major in m (the reduction index), so the MFMA fragments (8 consecutive m
// of one column per lane) are column reads of the staged tiles:
//   * each 32-row stage of A (128 columns n) and B (128 columns c) is loaded as f32 (16-byte row
//     segments, coalesced), split in registers and written as limb images [limb][32 m][128 cols]
//     bf16 (8-byte stores of 4 columns; the 8-byte unit u of row m sits at u ^ 8 (m & 3));
//   * fragments come back with ds_read_b64_tr_b16 (the gfx950 transposing LDS read): a 16-lane
//     group reads a 4 m x 16 column block and lane i receives column i's four m values; two reads
//     give the 8 m of a 32x32x16 operand.  The XOR makes both the stores and the transposed reads
//     bank-conflict free;
//   * 128 x 128 output tile per workgroup, 4 waves (one per SIMD) of 64 x 64; register-staged
//     prefetch of stage t+2 while stage t computes, two LDS buffers, one barrier per stage; the
//     split / image writes of stage t+1 and the loads of stage t+2 are spread between stage t's
//     MFMA blocks;
//     persistent workgroups over XCD-contiguous tile ranges (column tiles of one (n, s, z) adjacent:
//     the A rows stay in that XCD's L2).
// Kernel forms (all bitwise equal on the same slices; tests/test_gpu_gemm.py):
//   * gemm_tn_ring_kernel<RA> - the default: RA x 128 tiles on 8 waves (RA = 256 for R % 256 == 0:
//     dW1, dW2; 128 otherwise: dW3), 16-row stages in a 3-deep LDS ring, each stage's fragments read
//     before the barrier that opens it, side work and next-stage reads placed in the MFMA shadows
//     (sched_group_barrier);
//   * with LGX_TN_RING=0: gemm_tn_ws_kernel<128> for 128-row tiles (producer waves stage and split,
//     consumer waves read fragments and issue MFMAs; LGX_TN_WS=0: gemm_tn_x3_kernel<4>) and
//     gemm_tn_x3_kernel<8>, the two-buffer form described above, for 256-row tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "lgx_internal.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float fx2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TT = 128;                   // output tile columns (c); rows (n): RA = 128 | 256
constexpr int TK = 32;                    // rows m per stage

// NWV = 4: 128 x 128 tile, 2 x 2 waves (one per SIMD); NWV = 8: 256 x 128 tile, 4 x 2 waves (two
// per SIMD: one wave's split VALU and LDS traffic overlap the other's MFMAs; half the staged B
// bytes per MFMA)
template <int NWV>
struct TC {
  static constexpr int RA = NWV == 8 ? 256 : 128;    // A image width (output rows n per tile)
  static constexpr int PT = 64 * NWV;
  static constexpr int IMGA = 3 * TK * RA * 2;       // A limb image per stage (24 | 48 KB)
  static constexpr int IMGB = 3 * TK * TT * 2;       // B limb image (24 KB)
  static constexpr int STAGE = IMGA + IMGB;
  static constexpr int AQ = RA / 4;                  // A column quads per row
  static constexpr int AR = TK * AQ / PT;            // staged A rows per thread (4)
  static constexpr int BR = TK * (TT / 4) / PT;      // staged B rows per thread (4 | 2)
  static constexpr int AROW = TK / AR;               // thread row groups (8 | 8)
  static constexpr int CS = AROW * AQ * 16;          // column-sum scratch: [row group][column quad] float4
  static constexpr int LDS = 2 * STAGE + CS;         // two buffers (96 | 144 KB) + 4 | 8 KB
  static_assert(AR == 4 && (BR == 4 || BR == 2), "staging layout");
};

struct TnArgs {
  int64_t Ms;            // rows per slice (% 32 == 0)
  int32_t R, Cc, S, batch;
  const float* A;
  int64_t lda, sa;
  const float* B;
  int64_t ldb, sb;
  float* C;
  int64_t ldc;
  float* colsum;         // [batch][S][R] per-slice column sums of A, or null
  int32_t rt, ct, tiles;
};

__device__ __forceinline__ void split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  lgx_split2(x0, x1, l0, l1, l2);   // (lgx_internal.h)
}

// staged row (m, column quad cq) of one operand into its limb image [limb][ROWS m][W cols]: split,
// three 8-byte stores; the 8-byte unit cq of row m sits at cq ^ 8 (m & 3)
template <int W, int ROWS = TK>
__device__ __forceinline__ void tn_store_row(char* img, const float4& v, int cq, int m) {
  uint2 l0, l1, l2;
#ifndef TN_NO_SPLIT
  split2(v.x, v.y, l0.x, l1.x, l2.x);
  split2(v.z, v.w, l0.y, l1.y, l2.y);
#else   // A/B: raw bits (wrong results; measures the split's VALU cost)
  l0 = make_uint2(__float_as_uint(v.x), __float_as_uint(v.y));
  l1 = make_uint2(__float_as_uint(v.z), __float_as_uint(v.w));
  l2 = l0;
#endif
  char* row = img + m * (W * 2) + ((cq ^ (8 * (m & 3))) << 3);
  *reinterpret_cast<uint2*>(row) = l0;
  *reinterpret_cast<uint2*>(row + ROWS * W * 2) = l1;
  *reinterpret_cast<uint2*>(row + 2 * ROWS * W * 2) = l2;
}

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// fragment of 32 columns (column block a: offset xa) for 16-k half s of an image W columns wide
// and ROWS rows per limb: limb l = two transposed reads (m = 16s + 8h + 0..3 and + 4..7)
template <int W, int ROWS = TK>
__device__ __forceinline__ bf16x8 tn_frag(const char* img, int l, int s, int lane_off, int xa) {
  const char* p = img + l * (ROWS * W * 2) + s * (16 * W * 2) + lane_off + xa;
  const s16x4 lo = tr_read(p), hi = tr_read(p + 4 * W * 2);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NWV>
__global__ void __launch_bounds__(64 * NWV, 1) gemm_tn_x3_kernel(TnArgs g) {
  using X = TC<NWV>;
  constexpr int RA = X::RA;
  extern __shared__ __attribute__((aligned(16))) char tlds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  // staging: A thread (column quad aq, rows 4 am .. 4 am + 3); B thread (bq, rows BR bm ..)
  const int aq = tid % X::AQ, am = tid / X::AQ;
  const int bq = tid & 31, bm = tid >> 5;
  // transposed-read lane offset: row 8h + q (+ 4 e), 8-byte unit 8 (a ^ q) + 4 gb + p
  const int q = (lane >> 2) & 3, p = lane & 3, gb = (lane >> 4) & 1;
  const int lane_a = (8 * h + q) * (RA * 2) + (4 * gb + p) * 8;
  const int lane_b = (8 * h + q) * (TT * 2) + (4 * gb + p) * 8;
  int xa[2], xb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    xa[i] = 64 * ((2 * wm + i) ^ q);
    xb[i] = 64 * ((2 * wn + i) ^ q);
  }
  const int xcd = blockIdx.x & 7;
  const int32_t stride = gridDim.x >> 3;
  const int32_t lo = (int32_t)((int64_t)xcd * g.tiles / 8), hi = (int32_t)((int64_t)(xcd + 1) * g.tiles / 8);
  const int nst = (int)(g.Ms / TK);
  const uint32_t sta = (uint32_t)(g.lda * 4), stb = (uint32_t)(g.ldb * 4);
  for (int32_t tile = lo + (blockIdx.x >> 3); tile < hi; tile += stride) {
    int32_t t = tile;
    const int ctile = t % g.ct;
    t /= g.ct;
    const int ntile = t % g.rt;
    t /= g.rt;
    const int s = t % g.S;
    const int z = t / g.S;
    const int64_t m0 = (int64_t)s * g.Ms;
    const char* Ab = reinterpret_cast<const char*>(g.A + z * g.sa + m0 * g.lda + ntile * RA);
    const char* Bb = reinterpret_cast<const char*>(g.B + z * g.sb + m0 * g.ldb + ctile * TT);
    const uint32_t oa = (4 * am) * sta + aq * 16, ob = (X::BR * bm) * stb + bq * 16;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    float4 sa[4], sb[X::BR];
#pragma unroll
    for (int i = 0; i < 4; ++i) sa[i] = *reinterpret_cast<const float4*>(Ab + oa + i * sta);
#pragma unroll
    for (int i = 0; i < X::BR; ++i) sb[i] = *reinterpret_cast<const float4*>(Bb + ob + i * stb);
    // column sums of this thread's staged A rows (column quad aq), for the first column tile of an
    // (n, s, z) only; cw = 1 while the staged stage is a real one (the last stages re-load)
    const bool csum = g.colsum != nullptr && ctile == 0;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    auto cs_add = [&](const float4& v, float w) {
      cs.x = fmaf(v.x, w, cs.x);
      cs.y = fmaf(v.y, w, cs.y);
      cs.z = fmaf(v.z, w, cs.z);
      cs.w = fmaf(v.w, w, cs.w);
    };
    __syncthreads();   // (previous tile's last reads of buffer 0 are done)
#pragma unroll
    for (int i = 0; i < 4; ++i) cs_add(sa[i], 1.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) tn_store_row<RA>(tlds, sa[i], aq, 4 * am + i);
#pragma unroll
    for (int i = 0; i < X::BR; ++i) tn_store_row<TT>(tlds + X::IMGA, sb[i], bq, X::BR * bm + i);
    if (nst > 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sa[i] = *reinterpret_cast<const float4*>(Ab + oa + TK * sta + i * sta);
#pragma unroll
      for (int i = 0; i < X::BR; ++i) sb[i] = *reinterpret_cast<const float4*>(Bb + ob + TK * stb + i * stb);
    }
    __syncthreads();
#ifdef TN_CLOCK   // A/B instrumentation: per-stage s_memtime stamps of workgroup 0's first tile into g.C
    uint64_t* clk = (blockIdx.x == 0 && lane == 0 && tile == lo)
                        ? reinterpret_cast<uint64_t*>(g.C + (int64_t)g.batch * g.S * g.R * g.ldc)   // past the output
                        : nullptr;
#define TN_STAMP(e) \
  if (clk && k < 32 && (wave & 3) == 0) clk[((wave >> 2) * 32 + k) * 4 + (e)] = __builtin_amdgcn_s_memtime()
#else
#define TN_STAMP(e)
#endif
    for (int k = 0; k < nst; ++k) {
      TN_STAMP(0);
      const char* ia = tlds + (k & 1) * X::STAGE;
      const char* ib = ia + X::IMGA;
      // stage k+1's split + image writes (into the other buffer, free since the last barrier) and
      // stage k+2's loads run between the MFMA blocks of stage k: unit u = one staged row of A
      // (u < 4) or B, its load re-issued right after its write (phase clock: serialised after the
      // MFMAs they took 1,240 + 350 of 3,710 cycles per stage).  Unconditional (a branch here
      // makes the compiler wait vmcnt(0) at every unit): the last stage writes the idle buffer,
      // the last two re-load stage nst-1.
      char* nb = tlds + ((k + 1) & 1) * X::STAGE;
      const int kl = min(k + 2, nst - 1);
      const uint32_t la = oa + kl * TK * sta, lb = ob + kl * TK * stb;
      const float cw = k + 1 < nst ? 1.f : 0.f;   // (stage k+1 exists)
      auto side = [&](int u) {
#ifdef TN_NO_SIDE
        return;
#endif
        if (u < 4) {
          cs_add(sa[u], cw);
          tn_store_row<RA>(nb, sa[u], aq, 4 * am + u);
          sa[u] = *reinterpret_cast<const float4*>(Ab + la + u * sta);
        } else if (u - 4 < X::BR) {
          tn_store_row<TT>(nb + X::IMGA, sb[u - 4], bq, X::BR * bm + u - 4);
          sb[u - 4] = *reinterpret_cast<const float4*>(Bb + lb + (u - 4) * stb);
        }
      };
      // 4 waves: the fragments of half 1 are read while half 0's MFMAs run (registers to spare at
      // one wave per SIMD); 8 waves: one half at a time (the other wave covers the read latency)
      constexpr int FB = NWV == 4 ? 2 : 1;
      bf16x8 fa[FB][2][3], fb[FB][2][3];
      auto read_half = [&](int hs) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int l = 0; l < 3; ++l) {
            fa[hs % FB][i][l] = tn_frag<RA>(ia, l, hs, lane_a, xa[i]);
            fb[hs % FB][i][l] = tn_frag<TT>(ib, l, hs, lane_b, xb[i]);
          }
      };
      read_half(0);
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        if (FB == 2 && hs == 0) read_half(1);
        if (FB == 1 && hs == 1) read_half(1);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x16 c = acc[i][j];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][2], fb[hs % FB][j][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][1], fb[hs % FB][j][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][0], fb[hs % FB][j][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][1], fb[hs % FB][j][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][0], fb[hs % FB][j][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % FB][i][0], fb[hs % FB][j][0], c, 0, 0, 0);
            acc[i][j] = c;
            side(4 * hs + 2 * i + j);
            __builtin_amdgcn_sched_barrier(0);   // keep each unit between its MFMA blocks
          }
      }
      TN_STAMP(1);
      TN_STAMP(2);
      TN_STAMP(3);
      __syncthreads();
    }
    if (csum) {   // the 8 row groups' partial column sums, combined in a fixed order
      float4* scr = reinterpret_cast<float4*>(tlds + 2 * X::STAGE);
      scr[am * X::AQ + aq] = cs;
      __syncthreads();
      if (tid < X::AQ) {
        float4 t = scr[tid];
#pragma unroll
        for (int i = 1; i < X::AROW; ++i) {
          const float4 u = scr[i * X::AQ + tid];
          t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        *reinterpret_cast<float4*>(g.colsum + (int64_t)(z * g.S + s) * g.R + ntile * RA + 4 * tid) = t;
      }
    }
    // acc[i][j][e] = C[n0 + 32i + 8(e >> 2) + 4h + (e & 3)][c0 + 32j + r]: 32 lanes store one
    // 128-byte row segment per element
    float* Cb = g.C + ((int64_t)(z * g.S + s) * g.R + ntile * RA + wm * 64) * g.ldc;
    const int c0 = ctile * TT + wn * 64 + r;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + 32 * j;
      if (c >= g.Cc) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
          Cb[(int64_t)n * g.ldc + c] = acc[i][j][e];
        }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Warp-specialised form, used for the 128-row tiles (dW3 of the update; LGX_TN_WS=0 selects the
// 4-wave gemm_tn_x3_kernel<4> there, LGX_TN_WS=2 this form for the 256-row tiles too).  In the form
// above every wave both stages operands (global loads, the f32 -> limb split, LDS image writes) and
// issues MFMAs.  Here the roles are split between the two waves of each SIMD:
//   * consumers, waves 0-3 (one per SIMD, the older: they win issue arbitration): 32 WI x 128
//     output block each, an instruction stream of transposed fragment reads and MFMAs only - the
//     next B column block's fragments (and at j = 1 the next half's A fragments) are read under the
//     current block's 6 WI MFMAs;
//   * producers, waves 4-7: the global loads two stages ahead, the split and the limb-image writes
//     of the next stage, the column sums - in the consumers' MFMA gaps.
// Same LDS images (two stage buffers), one barrier per stage for all 8 waves, and the same products
// in the same order per output element: bitwise the results of gemm_tn_x3_kernel.
// Measured (round 6, isolated, half-GPU row slices, s_memtime per stage of workgroup 0):
//   * 128-row tiles (dW3, R = 128): 64.6 vs 69.2 us for the 4-wave kernel (S = 16), 36.4 vs 38.8 us (S = 32);
//   * 256-row tiles (dW1 / dW2): 122 vs 115-120 us (S = 16) - the producers are the bound: 4,877 cycles
//     per stage to stage 12,288 floats (4,824 with the consumers' MFMAs running, 2,726 without them)
//     against the consumers' 3,706 (96 MFMAs: 3,072-cycle floor).  The split VALU of a 256 x 128 tile
//     stage does not fit one wave per SIMD; the 8-wave kernel spreads it over both waves.
template <int RA>
struct TW {
  static constexpr int WI = RA / 128;                // 32-row A blocks per consumer wave (2 | 1)
  static constexpr int IMGA = 3 * TK * RA * 2;
  static constexpr int IMGB = 3 * TK * TT * 2;
  static constexpr int STAGE = IMGA + IMGB;
  static constexpr int AQ = RA / 4;                  // A column quads per row (64 | 32)
  static constexpr int AR = TK * AQ / 256;           // staged A rows per producer thread (8 | 4)
  static constexpr int BR = TK * (TT / 4) / 256;     // staged B rows per producer thread (4)
  static constexpr int AROW = 256 / AQ;              // producer row groups (4 | 8)
  static constexpr int CS = AROW * AQ * 16;          // column-sum scratch
  static constexpr int LDS = 2 * STAGE + CS;         // 148 KB | 100 KB
  static_assert(WI * 128 == RA && AR * AROW == TK && BR == 4, "layout");
};

// Tile coordinates of persistent tile `tile` (column tiles of one (n, s, z) adjacent)
struct TnTile {
  int ctile, ntile, s, z;
};
__device__ __forceinline__ TnTile tn_tile(const TnArgs& g, int32_t t) {
  TnTile T;
  T.ctile = t % g.ct;
  t /= g.ct;
  T.ntile = t % g.rt;
  t /= g.rt;
  T.s = t % g.S;
  T.z = t / g.S;
  return T;
}

// The two roles run separate loops over the same tiles and stages (so that neither role's
// registers are live in the other's: the accumulators and the staging registers would not fit one
// wave together) with the same barrier sequence: per tile one after the first stage's image
// writes, one per stage, and one before the column sums are combined.
template <int RA>
__device__ __forceinline__ void tn_ws_consumer(const TnArgs& g, char* tlds, int wave, int lane, int32_t lo, int32_t hi,
                                               int32_t stride, int nst) {
  using X = TW<RA>;
  constexpr int WI = X::WI;
  const int r = lane & 31, h = lane >> 5;
  const int q = (lane >> 2) & 3, p = lane & 3, gb = (lane >> 4) & 1;
  const int lane_a = (8 * h + q) * (RA * 2) + (4 * gb + p) * 8;
  const int lane_b = (8 * h + q) * (TT * 2) + (4 * gb + p) * 8;
  int xa[WI], xb[4];
#pragma unroll
  for (int i = 0; i < WI; ++i) xa[i] = 64 * ((WI * wave + i) ^ q);
#pragma unroll
  for (int j = 0; j < 4; ++j) xb[j] = 64 * (j ^ q);
  for (int32_t tile = lo + (blockIdx.x >> 3); tile < hi; tile += stride) {
    const TnTile T = tn_tile(g, tile);
    f32x16 acc[WI][4];
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    __syncthreads();   // stage 0 written
#ifdef TN_WS_CLOCK   // A/B instrumentation: s_memtime at each stage's start / end (after / before its
                     // barriers) of workgroup 0's first tile, waves 0 and 4, into the tail of g.C
    uint64_t* clk = (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && tile == lo + (blockIdx.x >> 3) && wave == 0)
                        ? reinterpret_cast<uint64_t*>(g.C + (int64_t)g.batch * g.S * g.R * g.ldc) : nullptr;
#endif
    for (int k = 0; k < nst; ++k) {
#ifdef TN_WS_CLOCK
      if (clk && k < 32) clk[k * 4 + 0] = __builtin_amdgcn_s_memtime();
#endif
      const char* ia = tlds + (k & 1) * X::STAGE;
      const char* ib = ia + X::IMGA;
      bf16x8 fa[2][WI][3], fb[2][3];
      auto read_a = [&](int buf, int hs) {
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int l = 0; l < 3; ++l) fa[buf][i][l] = tn_frag<RA>(ia, l, hs, lane_a, xa[i]);
      };
      auto read_b = [&](int buf, int hs, int j) {
#pragma unroll
        for (int l = 0; l < 3; ++l) fb[buf][l] = tn_frag<TT>(ib, l, hs, lane_b, xb[j]);
      };
      read_a(0, 0);
      read_b(0, 0, 0);
#pragma unroll
      for (int hs = 0; hs < 2; ++hs)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cb = (4 * hs + j) & 1;   // B fragment buffer of (hs, j)
          // the next block's fragments under this block's MFMAs
          if (j < 3) read_b(cb ^ 1, hs, j + 1);
          else if (hs == 0) read_b(cb ^ 1, 1, 0);
          if (hs == 0 && j == 1) read_a(1, 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < WI; ++i) {
            f32x16 c = acc[i][j];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][2], fb[cb][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][1], fb[cb][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][0], fb[cb][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][1], fb[cb][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][0], fb[cb][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs][i][0], fb[cb][0], c, 0, 0, 0);
            acc[i][j] = c;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#ifdef TN_WS_CLOCK
      if (clk && k < 32) clk[k * 4 + 1] = __builtin_amdgcn_s_memtime();
#endif
      __syncthreads();   // stage k read; stage k+1 written
    }
    if (g.colsum != nullptr && T.ctile == 0) __syncthreads();   // (the producers' column-sum exchange)
    // acc[i][j][e] = C[n0 + 32 i + 8 (e >> 2) + 4 h + (e & 3)][c0 + 32 j + r]
    float* Cb = g.C + ((int64_t)(T.z * g.S + T.s) * g.R + T.ntile * RA + wave * 32 * WI) * g.ldc;
    const int c0 = T.ctile * TT + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 32 * j;
      if (c >= g.Cc) continue;
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
          Cb[(int64_t)n * g.ldc + c] = acc[i][j][e];
        }
    }
  }
}

// Producer: the staged rows of TWO stages in registers (loads two stages ahead of their image
// writes: measured alone, the producers with one stage in flight took as long per stage as the
// consumers' MFMA floor - latency-bound on the global loads)
template <int RA>
__device__ __forceinline__ void tn_ws_producer(const TnArgs& g, char* tlds, int pt, int32_t lo, int32_t hi,
                                               int32_t stride, int nst) {
  using X = TW<RA>;
  const int aq = pt % X::AQ, am = pt / X::AQ;   // A thread: column quad aq, rows AR am ..
  const int bq = pt & 31, bm = pt >> 5;         // B thread: column quad bq, rows 4 bm ..
  const uint32_t sta = (uint32_t)(g.lda * 4), stb = (uint32_t)(g.ldb * 4);
  for (int32_t tile = lo + (blockIdx.x >> 3); tile < hi; tile += stride) {
    const TnTile T = tn_tile(g, tile);
    const int64_t m0 = (int64_t)T.s * g.Ms;
    const char* Ab = reinterpret_cast<const char*>(g.A + T.z * g.sa + m0 * g.lda + T.ntile * RA);
    const char* Bb = reinterpret_cast<const char*>(g.B + T.z * g.sb + m0 * g.ldb + T.ctile * TT);
    const uint32_t oa = (X::AR * am) * sta + aq * 16, ob = (X::BR * bm) * stb + bq * 16;
    const bool csum = g.colsum != nullptr && T.ctile == 0;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 sa[2][X::AR], sb[2][X::BR];   // register ring of two stages
    auto load = [&](float4 (&ra)[X::AR], float4 (&rb)[X::BR], int k) {
      const uint32_t la = oa + min(k, nst - 1) * TK * sta, lb = ob + min(k, nst - 1) * TK * stb;
#pragma unroll
      for (int i = 0; i < X::AR; ++i) ra[i] = *reinterpret_cast<const float4*>(Ab + la + i * sta);
#pragma unroll
      for (int i = 0; i < X::BR; ++i) rb[i] = *reinterpret_cast<const float4*>(Bb + lb + i * stb);
    };
    // stage k (registers ra / rb) into buffer k & 1; each staged row's reload for stage k + 2 right
    // after its write (past the last stage: re-loads of stage nst - 1, never written)
    auto write_reload = [&](float4 (&ra)[X::AR], float4 (&rb)[X::BR], int k) {
      char* nb = tlds + (k & 1) * X::STAGE;
      const int kl = min(k + 2, nst - 1);
      const uint32_t la = oa + kl * TK * sta, lb = ob + kl * TK * stb;
#pragma unroll
      for (int i = 0; i < X::AR; ++i) {
        cs.x += ra[i].x; cs.y += ra[i].y; cs.z += ra[i].z; cs.w += ra[i].w;
        tn_store_row<RA>(nb, ra[i], aq, X::AR * am + i);
        ra[i] = *reinterpret_cast<const float4*>(Ab + la + i * sta);
      }
#pragma unroll
      for (int i = 0; i < X::BR; ++i) {
        tn_store_row<TT>(nb + X::IMGA, rb[i], bq, X::BR * bm + i);
        rb[i] = *reinterpret_cast<const float4*>(Bb + lb + i * stb);
      }
    };
    load(sa[0], sb[0], 0);
    load(sa[1], sb[1], 1);
    // stage 0 into buffer 0 (its readers finished at the previous tile's last barrier); stage 2 in
    // flight behind stage 1
    write_reload(sa[0], sb[0], 0);
    __syncthreads();   // stage 0 written
    // iteration k: stage k + 1 into the other buffer (its readers finished stage k - 1 at the last
    // barrier) from ring entry (k + 1) & 1, which then loads stage k + 3
#ifdef TN_WS_CLOCK
    uint64_t* clk = (blockIdx.x == 0 && (pt & 63) == 0 && tile == lo + (blockIdx.x >> 3) && pt == 0)
                        ? reinterpret_cast<uint64_t*>(g.C + (int64_t)g.batch * g.S * g.R * g.ldc) : nullptr;
#define TN_PSTAMP(kk, e) if (clk && (kk) < 32) clk[(kk) * 4 + (e)] = __builtin_amdgcn_s_memtime()
#else
#define TN_PSTAMP(kk, e)
#endif
    for (int k = 0; k < nst; k += 2) {
      TN_PSTAMP(k, 2);
      if (k + 1 < nst) write_reload(sa[1], sb[1], k + 1);
      TN_PSTAMP(k, 3);
      __syncthreads();   // stage k read; stage k+1 written
      if (k + 1 < nst) {
        TN_PSTAMP(k + 1, 2);
        if (k + 2 < nst) write_reload(sa[0], sb[0], k + 2);
        TN_PSTAMP(k + 1, 3);
        __syncthreads();
      }
    }
    if (csum) {   // the AROW row groups' partial column sums, combined in a fixed order
      float4* scr = reinterpret_cast<float4*>(tlds + 2 * X::STAGE);
      scr[am * X::AQ + aq] = cs;
      __syncthreads();
      if (pt < X::AQ) {
        float4 v = scr[pt];
#pragma unroll
        for (int i = 1; i < X::AROW; ++i) {
          const float4 u = scr[i * X::AQ + pt];
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        *reinterpret_cast<float4*>(g.colsum + (int64_t)(T.z * g.S + T.s) * g.R + T.ntile * RA + 4 * pt) = v;
      }
    }
  }
}

template <int RA>
__global__ void __launch_bounds__(512, 1) gemm_tn_ws_kernel(TnArgs g) {
  extern __shared__ __attribute__((aligned(16))) char tlds[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xcd = blockIdx.x & 7;
  const int32_t stride = gridDim.x >> 3;
  const int32_t lo = (int32_t)((int64_t)xcd * g.tiles / 8), hi = (int32_t)((int64_t)(xcd + 1) * g.tiles / 8);
  const int nst = (int)(g.Ms / TK);
  if (wave < 4)
    tn_ws_consumer<RA>(g, tlds, wave, tid & 63, lo, hi, stride, nst);
  else
    tn_ws_producer<RA>(g, tlds, tid & 255, lo, hi, stride, nst);
}


// ---------------------------------------------------------------------------------------------
// Ring form of the 256-row tiles (the default for R % 256 == 0; LGX_TN_RING=0 selects
// gemm_tn_x3_kernel<8>).  Measured on gemm_tn_x3_kernel<8> (dW1 at the half-GPU slices, isolated):
// 118 us as built, 112 us without the split, 94 us with no staging at all (stale LDS) - against a
// 61-70 us MFMA floor: the fragment reads that open every 32-row stage after its barrier are exposed
// with both waves of a SIMD waiting on them at once.  This form stages 16-row images in a 3-deep LDS
// ring (36 KB per stage): stage k+1 is complete one barrier before it is computed, so each wave reads
// stage k+1's fragments right after its last MFMA of stage k and before that barrier - the read
// latency overlaps the barrier wait instead of following it.  Per stage and wave: 24 MFMAs (a 64 x 64
// block of 2 x 2 accumulators, one 16-k step) with the staging of stage k+2 (2 A rows + 1 B row per
// thread: split, limb-image writes) between the MFMA blocks; the global loads run two stages ahead in
// a register ring.  Same products in the same order per output element: bitwise the weight gradients
// of gemm_tn_x3_kernel.
// Measured (round 6, isolated, kbench tn, 2 alternations): half-GPU slices (S = 16) dW1 111-112 us
// vs 117, dW2 107-108 vs 114; S = 32 equal (75-76, 69-71); the full update 10.02 vs 10.06 ms (the
// dW launches run beside dA there).  Per-stage clock (s_memtime, workgroup 0, waves 0 and 4 of SIMD
// 0): 2,500 cycles per 16-row stage against the SIMD's 1,536 MFMA cycles - the later wave's MFMA
// region 1,915 (the side work's issue), the write wait 90, the 24 fragment-read issues 250 and the
// barrier 250; the older wave waits 650 at the barrier.  The loop must stay branch-free with the
// register ring in fixed registers (an `if` on the second half made the compiler copy the ring at the
// back edge behind vmcnt waits: 3 % slower than the old kernel).
constexpr int TR = 16;   // rows per ring stage

template <int RA_>
struct TRing {
  static constexpr int RA = RA_;
  static constexpr int WI = RA / 128;                // 32-row accumulator blocks per wave (wave: 32 WI x 64)
  static constexpr int AQ = RA / 4;                  // column quads of an A row
  static constexpr int AR = RA / 128;                // A rows per thread and stage
  static constexpr int IMGA = 3 * TR * RA * 2;       // 24 | 12 KB
  static constexpr int IMGB = 3 * TR * TT * 2;       // 12 KB
  static constexpr int STAGE = IMGA + IMGB;          // 36 | 24 KB
  static constexpr int NB = 3;                       // ring depth
  static constexpr int CS = 512 * 16;                // column-sum scratch: [row group][column quad] float4
  static constexpr int LDS = NB * STAGE + CS;        // 116 | 80 KB
};

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int RA>   // 256: dW1 / dW2 (wave blocks of 64 x 64); 128: wave blocks of 32 x 64
__global__ void __launch_bounds__(512, 1) gemm_tn_ring_kernel(TnArgs g) {
  using X = TRing<RA>;
  constexpr int WI = X::WI, AR = X::AR, AQ = X::AQ;
  extern __shared__ __attribute__((aligned(16))) char tlds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int q = (lane >> 2) & 3, p = lane & 3, gb = (lane >> 4) & 1;
  const int lane_a = (8 * h + q) * (RA * 2) + (4 * gb + p) * 8;
  const int lane_b = (8 * h + q) * (TT * 2) + (4 * gb + p) * 8;
  int xa[WI], xb[2];
#pragma unroll
  for (int i = 0; i < WI; ++i) xa[i] = 64 * ((WI * wm + i) ^ q);
#pragma unroll
  for (int j = 0; j < 2; ++j) xb[j] = 64 * ((2 * wn + j) ^ q);
  // staging: A thread = column quad aq of rows AR am .. AR am + AR - 1; B thread = column quad bq of row bm
  const int aq = tid % AQ, am = tid / AQ;
  const int bq = tid & 31, bm = tid >> 5;
  const int xcd = blockIdx.x & 7;
  const int32_t stride = gridDim.x >> 3;
  const int32_t lo = (int32_t)((int64_t)xcd * g.tiles / 8), hi = (int32_t)((int64_t)(xcd + 1) * g.tiles / 8);
  const int nst = (int)(g.Ms / TR);
  const uint32_t sta = (uint32_t)(g.lda * 4), stb = (uint32_t)(g.ldb * 4);
  for (int32_t tile = lo + (blockIdx.x >> 3); tile < hi; tile += stride) {
    int32_t t = tile;
    const int ctile = t % g.ct;
    t /= g.ct;
    const int ntile = t % g.rt;
    t /= g.rt;
    const int s = t % g.S;
    const int z = t / g.S;
    const int64_t m0 = (int64_t)s * g.Ms;
    const char* Ab = reinterpret_cast<const char*>(g.A + z * g.sa + m0 * g.lda + ntile * RA);
    const char* Bb = reinterpret_cast<const char*>(g.B + z * g.sb + m0 * g.ldb + ctile * TT);
    const uint32_t oa = (AR * am) * sta + aq * 16, ob = bm * stb + bq * 16;
    const bool csum = g.colsum != nullptr && ctile == 0;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 ra[2][AR], rb[2];          // register ring: stages k + 2 (slot k & 1) and k + 3
    auto load = [&](int slot, int k) {
      const int kc = min(k, nst - 1);   // (past the last stage: re-loads, never written as a stage)
      const uint32_t la = oa + kc * TR * sta, lb = ob + kc * TR * stb;
#pragma unroll
      for (int u = 0; u < AR; ++u) ra[slot][u] = *reinterpret_cast<const float4*>(Ab + la + u * sta);
      rb[slot] = *reinterpret_cast<const float4*>(Bb + lb);
    };
    f32x16 acc[WI][2];
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    bf16x8 fa[WI][3], fb[2][3];
    auto pre_a = [&](const char* ia, int i) {
#pragma unroll
      for (int l = 0; l < 3; ++l) fa[i][l] = tn_frag<RA, TR>(ia, l, 0, lane_a, xa[i]);
    };
    auto pre_b = [&](const char* ia, int j) {
#pragma unroll
      for (int l = 0; l < 3; ++l) fb[j][l] = tn_frag<TT, TR>(ia + X::IMGA, l, 0, lane_b, xb[j]);
    };
    auto prefetch = [&](const char* ia) {
#pragma unroll
      for (int i = 0; i < WI; ++i) pre_a(ia, i);
#pragma unroll
      for (int j = 0; j < 2; ++j) pre_b(ia, j);
    };
    __syncthreads();   // (the previous tile's readers of the ring are done)
    // prologue: stages 0 and 1 into ring buffers 0 and 1, stages 2 and 3 in flight
    load(0, 0);
    load(1, 1);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      char* wb = tlds + st * X::STAGE;
      const float cw = st < nst ? 1.f : 0.f;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        cs.x = fmaf(ra[st][i].x, cw, cs.x); cs.y = fmaf(ra[st][i].y, cw, cs.y);
        cs.z = fmaf(ra[st][i].z, cw, cs.z); cs.w = fmaf(ra[st][i].w, cw, cs.w);
        tn_store_row<RA, TR>(wb, ra[st][i], aq, AR * am + i);
      }
      tn_store_row<TT, TR>(wb + X::IMGA, rb[st], bq, bm);
      load(st, st + 2);
    }
    __syncthreads();
    prefetch(tlds);
#ifdef RING_CLOCK   // A/B instrumentation: per-stage s_memtime stamps of workgroup 0's first tile into g.C
    uint64_t* clk = (blockIdx.x == 0 && lane == 0 && tile == lo && (wave & 3) == 0)
                        ? reinterpret_cast<uint64_t*>(g.C + (int64_t)g.batch * g.S * g.R * g.ldc)
                        : nullptr;
#define RING_STAMP(e) \
  if (clk && k < 32) clk[((wave >> 2) * 32 + k) * 4 + (e)] = __builtin_amdgcn_s_memtime()
#else
#define RING_STAMP(e)
#endif
    uint32_t off_c = 0, off_w = 2 * X::STAGE;   // ring offsets of stage k (compute) and k + 2 (write)
    // stage k: MFMAs on the fragments prefetched before the last barrier; between the MFMA blocks the
    // images of stage k + 2 (ring slot SL) and the loads of stage k + 4; then stage k + 1's fragments
    auto step = [&](auto slot_c, int k) {
      constexpr int SL = decltype(slot_c)::value;
      RING_STAMP(0);
      char* wb = tlds + off_w;
      const uint32_t off_n = off_c == 2 * X::STAGE ? 0u : off_c + X::STAGE;   // stage k + 1
      const float cw = k + 2 < nst ? 1.f : 0.f;   // (stage k + 2 exists: else the idle buffer is written)
      auto side = [&](int u) {   // unit u < AR: A row u; u == AR: the B row and the next loads
        if (u < AR) {
          cs.x = fmaf(ra[SL][u].x, cw, cs.x); cs.y = fmaf(ra[SL][u].y, cw, cs.y);
          cs.z = fmaf(ra[SL][u].z, cw, cs.z); cs.w = fmaf(ra[SL][u].w, cw, cs.w);
          tn_store_row<RA, TR>(wb, ra[SL][u], aq, AR * am + u);
        } else if (u == AR) {
          tn_store_row<TT, TR>(wb + X::IMGA, rb[SL], bq, bm);
          load(SL, k + 4);
        }
      };
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
          acc[i][j] = c;
          side(2 * i + j);
          if (WI == 2 && i == 1 && j == 1) {   // the last block (no side unit): stage k + 1's block-0
            pre_a(tlds + off_n, 0);   // fragments, dead since block (1, 0), two reads per MFMA (104 /
            pre_b(tlds + off_n, 0);   // 101 vs 106 / 104 us for dW1 / dW2 at S = 16 with all 24 after it)
#pragma unroll
            for (int x = 0; x < 6; ++x) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            continue;
          }
          if (WI == 1 && j == 1) {   // the last block of a 32-row wave: its side unit and B block 0
            pre_b(tlds + off_n, 0);
#pragma unroll
            for (int x = 0; x < 6; ++x) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
              __builtin_amdgcn_sched_group_barrier(0x100 | 0x200, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            continue;
          }
          // the side unit spread over the block's MFMA shadows: per MFMA up to 4 VALU and one LDS
          // instruction (the compiler's own placement bunched them after the block: dW1 / dW2 at
          // S = 16 112.7 / 111.1 -> 107.8 / 105.4 us; 2 VALU per MFMA 113 / 112, 6 VALU 108 / 107)
#pragma unroll
          for (int x = 0; x < 6; ++x) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
            __builtin_amdgcn_sched_group_barrier(0x100 | 0x200, 1, 0);   // LDS read / write
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      // this stage's image writes complete before the barrier (the prefetch reads below may stay in
      // flight across it: their registers are waited for at the next stage's first MFMA)
      RING_STAMP(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      RING_STAMP(2);
      off_c = off_n;
      off_w = off_w == 2 * X::STAGE ? 0u : off_w + X::STAGE;
      // the rest of stage k + 1's fragments (complete since the last barrier; after the last stage
      // a stale buffer, unused - no branch in the loop).  Without the group schedule, issuing the
      // block-0 fragments as their registers die (A after MFMA block (0, 1), B after (1, 0))
      // lengthened the MFMA region by 130-190 cycles per stage and the kernel by 6 %
      pre_a(tlds + off_n, WI - 1);
      pre_b(tlds + off_n, 1);
      RING_STAMP(3);
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);   // (no MFMA of stage k + 1 above the barrier)
    };
    for (int k = 0; k < nst; k += 2) {   // (nst = Ms / 16 is even: slots 0 and 1 stay in their registers)
      step(std::integral_constant<int, 0>{}, k);
      step(std::integral_constant<int, 1>{}, k + 1);
    }
    if (csum) {   // the row groups' partial column sums, combined in a fixed order
      constexpr int NG = 512 / AQ;   // 8 | 16 row groups
      float4* scr = reinterpret_cast<float4*>(tlds + X::NB * X::STAGE);
      scr[am * AQ + aq] = cs;
      __syncthreads();
      if (tid < AQ) {
        float4 v = scr[tid];
#pragma unroll
        for (int i = 1; i < NG; ++i) {
          const float4 u = scr[i * AQ + tid];
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        *reinterpret_cast<float4*>(g.colsum + (int64_t)(z * g.S + s) * g.R + ntile * RA + 4 * tid) = v;
      }
    }
    // acc[i][j][e] = C[n0 + 32i + 8(e >> 2) + 4h + (e & 3)][c0 + 32j + r]
    float* Cb = g.C + ((int64_t)(z * g.S + s) * g.R + ntile * RA + wm * 32 * WI) * g.ldc;
    const int c0 = ctile * TT + wn * 64 + r;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + 32 * j;
      if (c >= g.Cc) continue;
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
          Cb[(int64_t)n * g.ldc + c] = acc[i][j][e];
        }
    }
  }
}

}  // namespace

extern "C" int lgx_gemm_tn(const lgx_gemm_tn_args* args, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_gemm_tn: null args");
  const lgx_gemm_tn_args& a = *args;
  if (!a.A || !a.B || !a.C || a.M <= 0 || a.slices <= 0 || a.M % a.slices || (a.M / a.slices) % TK || a.R <= 0 ||
      a.R % TT || a.Cc <= 0 || a.batch <= 0 || a.lda < a.R || a.ldb < (a.Cc + TT - 1) / TT * TT || a.ldc < a.Cc ||
      a.lda % 4 || a.ldb % 4 || a.sa % 4 || a.sb % 4 || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15))
    return lgx_fail(LGX_EINVAL,
                    "lgx_gemm_tn: bad args (M / slices % 32, R % 128, ldb >= Cc rounded up to 128, 16-byte aligned "
                    "A/B rows)");
  if ((a.M / a.slices + TK) * std::max(a.lda, a.ldb) * 4 >= (1ll << 32))
    return lgx_fail(LGX_EINVAL, "lgx_gemm_tn: row slice too large for 32-bit offsets");
  TnArgs g;
  g.Ms = a.M / a.slices;
  g.R = a.R;
  g.Cc = a.Cc;
  g.S = a.slices;
  g.batch = a.batch;
  g.A = a.A;
  g.lda = a.lda;
  g.sa = a.sa;
  g.B = a.B;
  g.ldb = a.ldb;
  g.sb = a.sb;
  g.C = a.C;
  g.ldc = a.ldc;
  g.colsum = a.colsum;
  if (a.colsum && ((uintptr_t)a.colsum & 15)) return lgx_fail(LGX_EINVAL, "lgx_gemm_tn: colsum must be 16-byte aligned");
  // 256-row tiles (8 waves) when R allows, else 128-row tiles; the ring form for both (LGX_TN_RING=0,
  // read per call for same-process A/B: the warp-specialised kernel for 128-row tiles - LGX_TN_WS=0:
  // the 4-wave gemm_tn_x3_kernel<4> - and gemm_tn_x3_kernel<8> for 256-row tiles - LGX_TN_WS=2: the
  // warp-specialised kernel)
  const char* wsv = getenv("LGX_TN_WS");
  const int wsm = wsv && *wsv ? atoi(wsv) : 1;
  const int nwv = a.R % 256 == 0 ? 8 : 4;
  const int RA = nwv == 8 ? 256 : 128;
  const char* rgv = getenv("LGX_TN_RING");
  const bool ringv = !(rgv && rgv[0] == '0') && (a.M / a.slices) % TR == 0;
  const bool ring = ringv && RA == 256, ring128 = ringv && RA == 128;
  const bool ws = !ringv && (RA == 128 ? wsm != 0 : wsm == 2);
  g.rt = a.R / RA;
  g.ct = (a.Cc + TT - 1) / TT;
  const int64_t tiles = (int64_t)g.rt * g.ct * a.slices * a.batch;
  if (tiles >= (1ll << 31) / 8) return lgx_fail(LGX_EINVAL, "lgx_gemm_tn: too many tiles");
  g.tiles = (int32_t)tiles;
  static const bool attrs =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_x3_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TC<4>::LDS) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_x3_kernel<8>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TC<8>::LDS) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_ws_kernel<256>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TW<256>::LDS) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_ws_kernel<128>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TW<128>::LDS) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_ring_kernel<256>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TRing<256>::LDS) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_ring_kernel<128>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          TRing<128>::LDS) == hipSuccess;
  if (!attrs) return lgx_fail(LGX_EHIP, "lgx_gemm_tn: hipFuncSetAttribute (dynamic LDS) failed");
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t per_xcd = (tiles + 7) / 8;
  const int64_t wgs = 8 * std::min<int64_t>(per_xcd, std::max(1, cus / 8));
  if (ring)
    LGX_LAUNCH(gemm_tn_ring_kernel<256>, dim3((unsigned)wgs), dim3(512), TRing<256>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  else if (ring128)
    LGX_LAUNCH(gemm_tn_ring_kernel<128>, dim3((unsigned)wgs), dim3(512), TRing<128>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  else if (ws && RA == 256)
    LGX_LAUNCH(gemm_tn_ws_kernel<256>, dim3((unsigned)wgs), dim3(512), TW<256>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  else if (ws)
    LGX_LAUNCH(gemm_tn_ws_kernel<128>, dim3((unsigned)wgs), dim3(512), TW<128>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  else if (nwv == 8)
    LGX_LAUNCH(gemm_tn_x3_kernel<8>, dim3((unsigned)wgs), dim3(512), TC<8>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  else
    LGX_LAUNCH(gemm_tn_x3_kernel<4>, dim3((unsigned)wgs), dim3(256), TC<4>::LDS, reinterpret_cast<hipStream_t>(stream), g);
  return lgx_hip_status("lgx_gemm_tn");
}
