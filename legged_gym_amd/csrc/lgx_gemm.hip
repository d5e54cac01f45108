// Hand-written f32 GEMMs of the PPO update with their epilogues fused (gfx950,
// v_mfma_f32_32x32x2_f32: exact f32, one rounding per product, 64 FLOP/clk/SIMD = the f32
// matrix peak).  They replace, per minibatch of rsl_rl PPO.update (legged_robot_config.py:
// 226-239), the library GEMM + separate epilogue passes of
//   forward  Y_k = ELU(Y_{k-1} W_k^T + b_k)                 (GEMM + lgx_bias_act), and
//   backward dZ_{k-1} = (dZ_k W_k) * ELU'(Y_{k-1}),  db_{k-1} = colsum(dZ_{k-1})
//                                                           (GEMM + lgx_elu_bwd_colsum),
// so every activation / gradient tile is written once, straight from the accumulators.
//
// Both are "NT" products C[z][m][n] = sum_k A[z][m][k] B[z][n][k] with K-contiguous rows on
// both sides (B = the nn.Linear weight for the forward, its transpose - prepared once per
// minibatch by lgx_copy2d - for the backward):
//   * workgroup = 4 waves, 128 x 128 output tile, wave = 64 x 64 = 2 x 2 accumulator tiles
//     (64 floats, 4 independent MFMA chains);
//   * K stages of 32: the A and B tiles (128 rows x 128 B each) are copied global -> LDS with
//     coalesced 16-byte loads, double-buffered (72 KB, 2 workgroups per CU), the next stage's
//     loads in flight during the current stage's MFMAs, one barrier per stage;
//   * 32x32x2 fragments: lane (r = l & 31, h = l >> 5) supplies A[row r][k] and B[k][col r]
//     for the MFMA's two k values.  One ds_read_b128 per operand gives a lane 4 consecutive k;
//     the k order is permuted (substep s of an 8-k group pairs k = s and 4 + s) identically
//     for A and B, so the sum is unchanged; rows padded by 16 B: conflict-free b128 reads;
//   * XCD-aware tile order: the tile index is split so that each of the 8 XCDs (workgroups
//     are dealt round-robin to XCDs) owns a contiguous range of tiles, n fastest, then the
//     batch index (actor / critic), then m: the A rows of one m-block (and, for the shared
//     layer-1 input, both networks) are reused out of one XCD's L2;
//   * epilogue in registers: bias + ELU, or ELU' (from the forward output) with the bias
//     gradient column sums reduced per 128-row tile in a fixed order (bitwise reproducible).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "lgx_gemm_common.h"
#include "lgx_internal.h"

#define LGX_STREAM(s) reinterpret_cast<hipStream_t>(s)

namespace {

constexpr int LDS_LD = BK + 4;      // row stride (floats): 16-B shift per row, conflict-free b128 reads
constexpr int TILE_FLOATS = BM * LDS_LD;

__device__ __forceinline__ float comp(const float4& q, int s) {
  return s == 0 ? q.x : s == 1 ? q.y : s == 2 ? q.z : q.w;
}

template <int NW>
__device__ __forceinline__ void stage_store(const Stage<NW>& st, float* __restrict__ la, float* __restrict__ lb, int K,
                                            int k0, int tid) {
  const int c = (tid & 7) * 4, r0 = tid >> 3;
  constexpr int RS = Cfg<NW>::RSTEP;
  if (k0 + BK <= K) {  // whole stage inside K (uniform)
#pragma unroll
    for (int i = 0; i < Cfg<NW>::NL; ++i) {
      *reinterpret_cast<float4*>(la + (r0 + RS * i) * LDS_LD + c) = st.a[i];
      *reinterpret_cast<float4*>(lb + (r0 + RS * i) * LDS_LD + c) = st.b[i];
    }
    return;
  }
  const bool in = k0 + c < K;
#pragma unroll
  for (int i = 0; i < Cfg<NW>::NL; ++i) {
    float4 va = st.a[i], vb = st.b[i];
    va.x = in ? va.x : 0.f; va.y = in ? va.y : 0.f; va.z = in ? va.z : 0.f; va.w = in ? va.w : 0.f;
    vb.x = in ? vb.x : 0.f; vb.y = in ? vb.y : 0.f; vb.z = in ? vb.z : 0.f; vb.w = in ? vb.w : 0.f;
    *reinterpret_cast<float4*>(la + (r0 + RS * i) * LDS_LD + c) = va;
    *reinterpret_cast<float4*>(lb + (r0 + RS * i) * LDS_LD + c) = vb;
  }
}

// MFMAs of one LDS stage.  Lane (r, h) reads 4 consecutive k of its row per ds_read_b128:
// k group g covers k = 8g .. 8g+7, lane half h holds 8g + 4h .. 8g + 4h + 3, and substep s of
// the group pairs (8g + s, 8g + 4 + s) - the same permutation for A and B.  The fragments of
// group g+1 are read while group g's MFMAs run (register double buffer).
template <int NW>
struct LdsFrag {
  float4 a[Cfg<NW>::WI], b[Cfg<NW>::WJ];
};

template <int NW>
__device__ __forceinline__ void frag_read(LdsFrag<NW>& f, const float* __restrict__ la, const float* __restrict__ lb,
                                          int wm, int wn, int r, int h, int g) {
  constexpr int WI = Cfg<NW>::WI, WJ = Cfg<NW>::WJ;
#pragma unroll
  for (int i = 0; i < WI; ++i)
    f.a[i] = *reinterpret_cast<const float4*>(la + (wm * 32 * WI + 32 * i + r) * LDS_LD + 8 * g + 4 * h);
#pragma unroll
  for (int j = 0; j < WJ; ++j)
    f.b[j] = *reinterpret_cast<const float4*>(lb + (wn * 32 * WJ + 32 * j + r) * LDS_LD + 8 * g + 4 * h);
}

template <int NW>
__device__ __forceinline__ void frag_mma(const LdsFrag<NW>& f, Acc<NW>& acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < Cfg<NW>::WI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg<NW>::WJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(f.a[i], s), comp(f.b[j], s), acc[i][j], 0, 0, 0);
}

template <int NW>
__device__ __forceinline__ void stage_mma(const float* __restrict__ la, const float* __restrict__ lb, int wm, int wn,
                                          int r, int h, Acc<NW>& acc) {
  LdsFrag<NW> f0, f1;
  frag_read<NW>(f0, la, lb, wm, wn, r, h, 0);
#pragma unroll
  for (int g = 0; g < BK / 8; g += 2) {
    frag_read<NW>(f1, la, lb, wm, wn, r, h, g + 1);
    __builtin_amdgcn_sched_barrier(0);
    frag_mma<NW>(f0, acc);
    __builtin_amdgcn_sched_barrier(0);
    if (g + 2 < BK / 8) frag_read<NW>(f0, la, lb, wm, wn, r, h, g + 2);
    __builtin_amdgcn_sched_barrier(0);
    frag_mma<NW>(f1, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Persistent workgroups: the tiles of XCD x (workgroups are dealt round-robin to the 8 XCDs)
// are the contiguous range [x T / 8, (x + 1) T / 8), n fastest, then the network, then m;
// workgroup w of the XCD takes its tiles w, w + W, ...  The first K stage of the next tile is
// loaded while the current tile's last stage and epilogue run.
template <int NW, int EPI>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 4 : 2) gemm_nt_kernel(GemmArgs g) {  // 2 workgroups per CU
  __shared__ __attribute__((aligned(16))) float lds[4 * TILE_FLOATS];  // 2 stages x (A tile, B tile): 72 KB
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave / Cfg<NW>::WGN, wn = wave % Cfg<NW>::WGN;
  const int ntn = g.N / BN;
  const int64_t total = ((g.M + BM - 1) / BM) * ntn * g.batch;
  const int xcd = blockIdx.x & 7;
  const int64_t wg_per_xcd = gridDim.x >> 3;     // grid is a multiple of 8
  const int64_t lo = xcd * total / 8, hi = (xcd + 1) * total / 8;
  int64_t tile = lo + (blockIdx.x >> 3);
  if (tile >= hi) return;
  const int K = g.K;
  const int nst = (K + BK - 1) / BK;

  TileId T = decode_tile(tile, ntn, g.batch);
  const int c = (tid & 7) * 4;
  RowOffs<NW> o;
  row_offs<NW>(o, g.lda, T.mt * BM, g.M, g.ldb, T.nt * BN, tid);
  Stage<NW> st;
  stage_load<NW>(st, g.A + T.z * g.sa, g.B + T.z * g.sb, o, K, 0, c);
  for (;;) {
    const int64_t next = tile + wg_per_xcd;
    const bool has_next = next < hi;
    const TileId Tn = decode_tile(has_next ? next : tile, ntn, g.batch);
    const float* A = g.A + T.z * g.sa;
    const float* B = g.B + T.z * g.sb;
    stage_store<NW>(st, lds, lds + TILE_FLOATS, K, 0, tid);
    __syncthreads();
    Acc<NW> acc;
#pragma unroll
    for (int i = 0; i < Cfg<NW>::WI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg<NW>::WJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    // double-buffered LDS stages: the global loads of stage t+1 are in flight while stage t's
    // MFMAs run; one barrier per stage
    for (int t = 0; t + 1 < nst; ++t) {
      float* cur = lds + (t & 1) * 2 * TILE_FLOATS;
      float* nxt = lds + ((t + 1) & 1) * 2 * TILE_FLOATS;
      stage_load<NW>(st, A, B, o, K, (t + 1) * BK, c);
      __builtin_amdgcn_sched_barrier(0);  // loads issued before the MFMAs they overlap
      if (g.prio) __builtin_amdgcn_s_setprio(1);
      stage_mma<NW>(cur, cur + TILE_FLOATS, wm, wn, r, h, acc);
      if (g.prio) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      stage_store<NW>(st, nxt, nxt + TILE_FLOATS, K, (t + 1) * BK, tid);
      __syncthreads();
    }
    {  // last stage: the next tile's stage 0 is in flight during its MFMAs and the epilogue
      float* cur = lds + ((nst - 1) & 1) * 2 * TILE_FLOATS;
      row_offs<NW>(o, g.lda, Tn.mt * BM, g.M, g.ldb, Tn.nt * BN, tid);
      stage_load<NW>(st, g.A + Tn.z * g.sa, g.B + Tn.z * g.sb, o, K, 0, c);
      __builtin_amdgcn_sched_barrier(0);
      if (g.prio) __builtin_amdgcn_s_setprio(1);
      stage_mma<NW>(cur, cur + TILE_FLOATS, wm, wn, r, h, acc);
      if (g.prio) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    }
    epilogue<NW, EPI>(g, acc, T, wm, wn, r, h);
    if (!has_next) break;
    tile = next;
    T = Tn;
  }
}


}  // namespace

// ---------------------------------------------------------------------------------------- copy2d
// dst[b][r][c] = src[b][r][c] (transpose = 0) or dst[b][c][r] = src[b][r][c] (transpose = 1),
// 32 x 32 tiles through LDS (odd row stride: conflict-free transposed reads).  Several jobs in
// one launch (the per-minibatch weight preparation of the fused GEMMs).
namespace {
struct Copy2dJobs {
  lgx_copy2d_job job[LGX_MAX_REDUCE_JOBS];
  int32_t tile_start[LGX_MAX_REDUCE_JOBS + 1];
  int32_t njobs;
};

__global__ void __launch_bounds__(256) copy2d_kernel(Copy2dJobs J) {
  __shared__ float t[32][33];
  int b = blockIdx.x, ji = 0;
  while (ji + 1 < J.njobs && b >= J.tile_start[ji + 1]) ++ji;
  const lgx_copy2d_job& jb = J.job[ji];
  const int local = b - J.tile_start[ji];
  const int tr = (jb.rows + 31) / 32, tc = (jb.cols + 31) / 32;
  const int bb = local / (tr * tc), rem = local % (tr * tc);
  const int r0 = (rem / tc) * 32, c0 = (rem % tc) * 32;
  const float* src = jb.src + (int64_t)bb * jb.src_bs;
  float* dst = jb.dst + (int64_t)bb * jb.dst_bs;
  const int x = threadIdx.x & 31, y = threadIdx.x >> 5;  // 8 rows of 32 per pass
  for (int yy = y; yy < 32; yy += 8) {
    const int rr = r0 + yy, cc = c0 + x;
    if (rr < jb.rows && cc < jb.cols) t[yy][x] = src[(int64_t)rr * jb.src_ld + cc];
  }
  __syncthreads();
  for (int yy = y; yy < 32; yy += 8) {
    if (jb.transpose) {
      const int cc = c0 + yy, rr = r0 + x;  // dst row = source column
      if (rr < jb.rows && cc < jb.cols) dst[(int64_t)cc * jb.dst_ld + rr] = t[x][yy];
    } else {
      const int rr = r0 + yy, cc = c0 + x;
      if (rr < jb.rows && cc < jb.cols) dst[(int64_t)rr * jb.dst_ld + cc] = t[yy][x];
    }
  }
}

// dst[r][0:width] = src[idx[r]][0:width], dst[r][width:dst_ld] = 0: one row per wave.
// dup > 0: blocks of `dup` rows are written twice, back to back (dst row (r / dup) * 2 dup +
// r % dup and `dup` rows further): one [2, dup, dst_ld] operand per block for a batched GEMM of
// two networks over the same rows.
__global__ void __launch_bounds__(256) gather_rows_padded_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                                 const int64_t* __restrict__ idx, int64_t rows,
                                                                 int32_t width, int32_t dst_ld, int64_t dup) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* s = src + idx[r] * width;
  const int64_t dr = dup > 0 ? (r / dup) * 2 * dup + r % dup : r;
  float* d = dst + dr * dst_ld;
  // four loads in flight per lane from clamped (always valid) columns, then the predicated stores
  // (a load under `c < width` compiled to one exposed round trip per column group)
  for (int c0 = 0; c0 < dst_ld; c0 += 256) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = s[min(c0 + 64 * i + lane, width - 1)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + 64 * i + lane;
      const float x = c < width ? v[i] : 0.f;
      if (c < dst_ld) {
        d[c] = x;
        if (dup > 0) d[dup * dst_ld + c] = x;
      }
    }
  }
}
}  // namespace

extern "C" int64_t lgx_gemm_partials_floats(int64_t M, int32_t N, int32_t batch) {
  return ((M + BM - 1) / BM) * (int64_t)N * batch;
}

extern "C" int lgx_gemm_nt(const lgx_gemm_args* args, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: null args");
  const lgx_gemm_args& a = *args;
  static const int default_algo = [] {
    const char* e = getenv("LGX_GEMM_ALGO");
    return e && e[0] == 'f' ? LGX_GEMM_ALGO_F32 : LGX_GEMM_ALGO_SPLIT_BF16;
  }();
  if (a.algo < 0 || a.algo > LGX_GEMM_ALGO_SPLIT_BF16) return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: bad algo");
  const int algo = a.algo == LGX_GEMM_ALGO_DEFAULT ? default_algo : a.algo;
  const bool presplit = algo == LGX_GEMM_ALGO_SPLIT_BF16 && a.Bs;   // B is not read
  const bool aligned = ((uintptr_t)a.A & 15) == 0 && a.lda % 4 == 0 && a.sa % 4 == 0 &&
                       (presplit || (((uintptr_t)a.B & 15) == 0 && a.ldb % 4 == 0 && a.sb % 4 == 0));
  if (!a.A || (!a.B && !presplit) || !a.C || a.M <= 0 || a.N <= 0 || a.N % BN || a.K <= 0 || a.K % 4 ||
      a.batch <= 0 || a.batch > 65535 || !aligned || a.lda < a.K || (!presplit && a.ldb < a.K) || a.ldc < a.N ||
      a.ldc > (1 << 22) || a.epi < 0 || a.epi > 3 || (a.epi == LGX_GEMM_BIAS_ELU && !a.bias) ||
      (a.epi == LGX_GEMM_DELU_COLSUM && (!a.Y || !a.partials)) || (a.epi == LGX_GEMM_DELU && !a.Y))
    return lgx_fail(LGX_EINVAL,
                    "lgx_gemm_nt: bad args (N % 128, K % 4, 16-byte aligned A/B rows, epilogue operands)");
  if (a.M * a.lda >= (1ll << 30) || (!presplit && (int64_t)a.N * a.ldb >= (1ll << 30)))
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: operand too large for 32-bit row offsets");
  if (algo == LGX_GEMM_ALGO_SPLIT_BF16 &&   // 16-byte epilogue vectors
      (((uintptr_t)a.C & 15) || a.ldc % 4 || a.sc % 4 || (a.bias && ((uintptr_t)a.bias & 15)) ||
       (a.Y && ((uintptr_t)a.Y & 15))))
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: split-bf16 path needs 16-byte aligned C / Y / bias rows");
  const int64_t tiles = ((a.M + BM - 1) / BM) * (a.N / BN) * a.batch;
  if (tiles > (1ll << 31) - 1) return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: too large");
  constexpr int prio = 1;   // s_setprio around the MFMA stages
  GemmArgs g{a.M, a.N, a.K, a.batch, a.epi, a.A, a.lda, a.sa, a.B, a.ldb, a.sb, a.C, a.ldc, a.sc, a.bias, a.Y,
             a.partials, prio, nullptr};
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t per_xcd = (tiles + 7) / 8;
  if (algo == LGX_GEMM_ALGO_SPLIT_BF16) return lgx_gemm_nt_split(a, cus, stream);
  if (a.epi == LGX_GEMM_DELU) return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: LGX_GEMM_DELU needs the split-bf16 algo");
  // persistent: 2 workgroups per CU (LDS-bound), a multiple of 8 (XCD tile ranges)
  const int64_t wgs = 8 * std::min<int64_t>(per_xcd, std::max(1, 2 * cus / 8));
  const dim3 grid((unsigned)wgs);
  const dim3 block(512);   // 8 waves per 128 x 128 tile
  if (a.epi == LGX_GEMM_BIAS_ELU) LGX_LAUNCH((gemm_nt_kernel<8, LGX_GEMM_BIAS_ELU>), grid, block, 0, LGX_STREAM(stream), g);
  else if (a.epi == LGX_GEMM_DELU_COLSUM)
    LGX_LAUNCH((gemm_nt_kernel<8, LGX_GEMM_DELU_COLSUM>), grid, block, 0, LGX_STREAM(stream), g);
  else LGX_LAUNCH((gemm_nt_kernel<8, LGX_GEMM_PLAIN>), grid, block, 0, LGX_STREAM(stream), g);
  return lgx_hip_status("lgx_gemm_nt");
}

extern "C" int lgx_copy2d(const lgx_copy2d_job* jobs, int32_t njobs, void* stream) {
  if (!jobs || njobs <= 0 || njobs > LGX_MAX_REDUCE_JOBS) return lgx_fail(LGX_EINVAL, "lgx_copy2d: bad job count");
  Copy2dJobs J;
  int64_t tiles = 0;
  J.njobs = njobs;
  for (int i = 0; i < njobs; ++i) {
    const lgx_copy2d_job& j = jobs[i];
    if (!j.src || !j.dst || j.rows <= 0 || j.cols <= 0 || j.batch <= 0 ||
        j.src_ld < j.cols || j.dst_ld < (j.transpose ? j.rows : j.cols))
      return lgx_fail(LGX_EINVAL, "lgx_copy2d: bad job");
    J.job[i] = j;
    J.tile_start[i] = (int32_t)tiles;
    tiles += (int64_t)j.batch * ((j.rows + 31) / 32) * ((j.cols + 31) / 32);
    if (tiles > (1 << 30)) return lgx_fail(LGX_EINVAL, "lgx_copy2d: too large");
  }
  J.tile_start[njobs] = (int32_t)tiles;
  hipLaunchKernelGGL(copy2d_kernel, dim3((unsigned)tiles), dim3(256), 0, LGX_STREAM(stream), J);
  return lgx_hip_status("lgx_copy2d");
}

extern "C" int lgx_ppo_gather_rows_padded(const float* src, float* dst, const int64_t* idx, int64_t rows,
                                          int32_t width, int32_t dst_ld, void* stream) {
  if (!src || !dst || !idx || rows <= 0 || width <= 0 || dst_ld < width)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_gather_rows_padded: bad args");
  hipLaunchKernelGGL(gather_rows_padded_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, LGX_STREAM(stream),
                     src, dst, idx, rows, width, dst_ld, (int64_t)0);
  return lgx_hip_status("lgx_ppo_gather_rows_padded");
}

extern "C" int lgx_ppo_gather_rows_padded_dup(const float* src, float* dst, const int64_t* idx, int64_t rows,
                                              int32_t width, int32_t dst_ld, int64_t block, void* stream) {
  if (!src || !dst || !idx || rows <= 0 || width <= 0 || dst_ld < width || block <= 0 || rows % block)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_gather_rows_padded_dup: bad args (rows % block)");
  hipLaunchKernelGGL(gather_rows_padded_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, LGX_STREAM(stream),
                     src, dst, idx, rows, width, dst_ld, block);
  return lgx_hip_status("lgx_ppo_gather_rows_padded_dup");
}
