// Pieces shared by the hand-written PPO-update GEMMs (lgx_gemm.hip: exact f32 MFMA;
// lgx_gemm_split.hip: split-bf16 evaluation): argument block, 128 x 128 tile / wave layouts,
// 16-byte register staging of f32 operand tiles, XCD-ordered tile decode and the fused
// epilogues (bias + ELU, ELU' + bias-gradient column sums) written from the accumulators.
// The 32x32 accumulator layout is the same for v_mfma_f32_32x32x2_f32 and
// v_mfma_f32_32x32x16_bf16 (C/D layout is dtype-independent on gfx950), so one epilogue serves
// both.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "lgx_internal.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128;     // rows per workgroup tile
constexpr int BN = 128;     // columns per workgroup tile

struct GemmArgs {
  int64_t M;
  int32_t N, K, batch, epi;
  const float* A;
  int64_t lda, sa;
  const float* B;
  int64_t ldb, sb;
  float* C;
  int64_t ldc, sc;
  const float* bias;
  const float* Y;
  float* partials;
  int32_t prio;   // raise the wave priority while issuing a stage's MFMAs (s_setprio)
  const uint16_t* Bs;   // split-bf16 path: B pre-split into bf16 limbs (or null)
};

__device__ __forceinline__ float elu_f(float x) { return lgx_elu(x); }
__device__ __forceinline__ float elu_grad_from_out(float y) { return y > 0.f ? 1.f : y + 1.f; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

constexpr int BK = 32;              // K per LDS stage
// Wave layouts of the 128 x 128 workgroup tile (template NW = waves per workgroup):
//   NW = 4: 2 x 2 waves of 64 x 64 (2 x 2 accumulator tiles of 32 x 32, 64 floats per lane);
//   NW = 8: 2 x 4 waves of 64 x 32 (2 x 1 tiles): half the accumulators per wave, 4 waves per
//           SIMD at 2 workgroups per CU, so one workgroup's epilogue and barriers are covered by
//           the other's MFMAs.
template <int NW>
struct Cfg {
  static constexpr int GT = 64 * NW;            // threads per workgroup
  static constexpr int WI = 2;                  // 32-row accumulator tiles per wave
  static constexpr int WJ = NW == 4 ? 2 : 1;    // 32-column accumulator tiles per wave
  static constexpr int WGN = BN / (32 * WJ);    // waves along N
  static constexpr int WGM = NW / WGN;          // waves along M
  static constexpr int NL = 1024 / GT;          // float4 per thread per operand per K stage
  static constexpr int RSTEP = GT / 8;          // row step between a thread's float4s
  static_assert(WGM * 32 * WI == BM, "wave grid covers the tile rows");
};

// One K stage of the global -> LDS copy: 128 rows x 32 k of A and of B (8 threads per 128-byte
// row segment: coalesced).  Thread t copies rows (t >> 3) + RSTEP i at columns c = (t & 7) * 4;
// its row offsets are 32-bit (the caller checks that every operand has < 2^30 floats: 32-bit
// byte offsets), so the loads address from the uniform base pointer (SGPRs) plus one VGPR
// offset instead of a 64-bit VGPR address per load.  k >= K is zero-filled.
template <int NW>
struct Stage {
  float4 a[Cfg<NW>::NL], b[Cfg<NW>::NL];
};
template <int NW>
struct RowOffs {
  uint32_t a[Cfg<NW>::NL], b[Cfg<NW>::NL];
};

template <int NW>
__device__ __forceinline__ void row_offs(RowOffs<NW>& o, int64_t lda, int64_t m_base, int64_t M, int64_t ldb,
                                         int n_base, int tid) {
#pragma unroll
  for (int i = 0; i < Cfg<NW>::NL; ++i) {
    const int row = (tid >> 3) + Cfg<NW>::RSTEP * i;
    const int64_t m = min(m_base + row, M - 1);  // rows past M load row M-1 (results discarded)
    o.a[i] = (uint32_t)(m * lda);
    o.b[i] = (uint32_t)((int64_t)(n_base + row) * ldb);
  }
}

template <int NW>
__device__ __forceinline__ void stage_load(Stage<NW>& st, const float* __restrict__ A, const float* __restrict__ B,
                                           const RowOffs<NW>& o, int K, int k0, int c) {
  // branch-free tail: past K, load the last valid float4 (zeroed in stage_store)
  const uint32_t kc = (uint32_t)min(k0 + c, K - 4);
  const char* Ab = reinterpret_cast<const char*>(A);
  const char* Bb = reinterpret_cast<const char*>(B);
#pragma unroll
  for (int i = 0; i < Cfg<NW>::NL; ++i) {  // 32-bit byte offsets: base (SGPR) + offset (VGPR)
    st.a[i] = *reinterpret_cast<const float4*>(Ab + (uint32_t)((o.a[i] + kc) * 4u));
    st.b[i] = *reinterpret_cast<const float4*>(Bb + (uint32_t)((o.b[i] + kc) * 4u));
  }
}

template <int NW>
using Acc = f32x16[Cfg<NW>::WI][Cfg<NW>::WJ];

struct TileId {
  int64_t mt;
  int nt, z;
};

__device__ __forceinline__ TileId decode_tile(int64_t tile, int ntn, int batch) {
  TileId t;
  t.nt = (int)(tile % ntn);
  const int64_t rest = tile / ntn;
  t.z = (int)(rest % batch);
  t.mt = rest / batch;
  return t;
}

// ---- epilogue: acc[i][j][e] is C[m0 + 32i + (e & 3) + 8(e >> 2) + 4h][n0 + 32j + r].
// Every store / load addresses a wave-uniform row pointer (SGPRs) plus ONE per-lane 32-bit
// byte offset (4h rows + r columns), so no per-row 64-bit addresses live in VGPRs; whole tiles
// (every tile when M % 128 == 0) store without row guards.
__device__ __forceinline__ int acc_row(int i, int e) { return 32 * i + (e & 3) + 8 * (e >> 2); }

template <typename T>
__device__ __forceinline__ T* at_bytes(T* p, uint32_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<typename std::conditional<std::is_const<T>::value, const char, char>::type*>(p) + off);
}

template <int NW, int EPI, bool FULL>
__device__ __forceinline__ void epilogue_rows(const GemmArgs& g, const Acc<NW>& acc, int64_t m0, int n0, int z, int r,
                                              int h, float (&cs)[Cfg<NW>::WJ]) {
  constexpr int WI = Cfg<NW>::WI, WJ = Cfg<NW>::WJ;
  float* C = g.C + z * g.sc + m0 * g.ldc + n0;
  const int64_t ldc = g.ldc;
  const int rows = (int)min<int64_t>(32 * WI, g.M - m0);
  const uint32_t lo = (uint32_t)((4 * h * ldc + r) * 4);  // this lane's byte offset from a row pointer
  if (EPI == LGX_GEMM_DELU_COLSUM) {
    const float* Y = g.Y + z * g.sc + m0 * g.ldc + n0;
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int e0 = 0; e0 < 16; e0 += 4) {   // 4 * WJ loads of Y in flight, then the stores
        float y[4][WJ];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < WJ; ++j) {
            const int rr = acc_row(i, e0 + e);
            y[e][j] = (FULL || rr + 4 * h < rows) ? *at_bytes(Y + rr * ldc + 32 * j, lo) : 0.f;
          }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < WJ; ++j) {
            const int rr = acc_row(i, e0 + e);
            const float d = acc[i][j][e0 + e] * elu_grad_from_out(y[e][j]);
            if (FULL || rr + 4 * h < rows) {
              *at_bytes(C + rr * ldc + 32 * j, lo) = d;
              cs[j] += d;
            }
          }
      }
  } else {
    float bj[WJ];
#pragma unroll
    for (int j = 0; j < WJ; ++j) bj[j] = EPI == LGX_GEMM_BIAS_ELU ? g.bias[(int64_t)z * g.N + n0 + 32 * j + r] : 0.f;
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          const int rr = acc_row(i, e);
          float v = acc[i][j][e];
          if (EPI == LGX_GEMM_BIAS_ELU) v = elu_f(v + bj[j]);
          if (FULL || rr + 4 * h < rows) *at_bytes(C + rr * ldc + 32 * j, lo) = v;
        }
  }
}

template <int NW, int EPI>
__device__ __forceinline__ void epilogue(const GemmArgs& g, const Acc<NW>& acc, const TileId& T, int wm, int wn, int r,
                                         int h) {
  constexpr int WI = Cfg<NW>::WI, WJ = Cfg<NW>::WJ, WGM = Cfg<NW>::WGM;
  const int64_t m0 = T.mt * BM + wm * 32 * WI;
  const int n0 = T.nt * BN + wn * 32 * WJ;
  float cs[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) cs[j] = 0.f;
  if (T.mt * BM + BM <= g.M) epilogue_rows<NW, EPI, true>(g, acc, m0, n0, T.z, r, h, cs);
  else if (m0 < g.M) epilogue_rows<NW, EPI, false>(g, acc, m0, n0, T.z, r, h, cs);
  if (EPI == LGX_GEMM_DELU_COLSUM) {
    // column sums: lane halves hold different rows of the same column, then the wave rows
    __shared__ float red[WGM][BN];  // [wave row][column within the tile]
#pragma unroll
    for (int j = 0; j < WJ; ++j) cs[j] += __shfl_xor(cs[j], 32);
    const int cl = wn * 32 * WJ;  // the wave's first column within the tile
    if (h == 0) {
#pragma unroll
      for (int j = 0; j < WJ; ++j) red[wm][cl + 32 * j + r] = cs[j];
    }
    __syncthreads();
    if (wm == 0 && h == 0) {
      float* P = g.partials + T.mt * ((int64_t)g.batch * g.N) + (int64_t)T.z * g.N;
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WGM; ++w) v += red[w][cl + 32 * j + r];   // fixed order
        P[n0 + 32 * j + r] = v;
      }
    }
  }
}

}  // namespace
