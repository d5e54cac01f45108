// Fused MLP forward on f32 MFMA (v_mfma_f32_16x16x4_f32: exact f32, one rounding per product,
// the f32 matrix peak of gfx950).  Used for
//   * the Go1 actuator network (UniNet core, go1.py:22-35,100-105): 30-128-128-128-3, tanh,
//     evaluated for decimation x N x 4 leg rows per env-step in ONE launch (the reference runs
//     4 legs x 4 substeps of small GEMMs plus 96 host<->device copies per env-step);
//   * rsl_rl ActorCritic inference in the rollout (obs-512-256-128-{12,1}, ELU): actor and
//     critic run in the SAME launch (blockIdx.y selects the network).
//
// Tiling (NW = 8 waves per workgroup for the policy nets, 4 for narrow nets; no barrier inside
// a layer's K loop):
//   * a row tile of BM = 16*RS rows stays in LDS across ALL layers: layer input and output
//     live at opposite ends of one activation region whose row strides are = 2 (mod 32), which
//     makes the MFMA A-fragment reads (16 rows x 2 k per 32-lane half) bank-conflict free;
//     HBM traffic is the input and output rows only;
//   * B fragments stream straight from the transposed weights W^T [in][out] (L2-resident,
//     16 consecutive columns per 4 k-rows = 4 x 64 B per load) into a double-buffered ring
//     of 8 VGPRs per lane, one group of k-steps ahead of the MFMAs consuming the other ring;
//   * wave w owns output column tiles w, w+NW, ... (16 columns each); a layer with TPW tiles
//     per wave processes G = 8/TPW k-steps per group, so every group is 8 B loads + 8*RS MFMAs;
//     8 waves on a 16-row tile halve each wave's column share (more waves in flight per
//     weight byte: 4096-row rollout 90 -> 86 us isolated, 3.85M -> 3.92M env-steps/s in situ);
//   * LDS is only the activation tile (<= 50 KB) -> 3-4 workgroups per CU hide the latency;
//   * grid-stride over row tiles (persistent when rows >> grid * BM).
#include <stdlib.h>

#include <algorithm>

#include "lgx_device.h"
#include "lgx_internal.h"

#define MLP_MAX_W 512
#define MLP_MAX_LAYERS 6
// register budget per lane of the fused kernel (no AGPR spill copies; 4 waves per SIMD fit)
#ifndef LGX_MLP_MAX_VGPR
#define LGX_MLP_MAX_VGPR 128
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct MlpArgs {
  const float* x;
  float* y;
  int64_t rows;
  int32_t nl;
  int32_t act;                      // 1 elu, 2 tanh
  int32_t dims[MLP_MAX_LAYERS + 1];
  const float* wt[MLP_MAX_LAYERS];  // [in][out]
  const float* b[MLP_MAX_LAYERS];
  const float* out_scale;           // optional per-output-column scale
};

struct MlpBatch {
  MlpArgs m[2];
};

LGX_DEV float activate(float x, int act) {
  if (act == 1) return lgx_elu(x);
  if (act == 2) return tanhf(x);
  return x;
}

__host__ __device__ inline int pad32(int n) { return (n + 31) & ~31; }
__host__ __device__ inline int pad16(int n) { return (n + 15) & ~15; }
__host__ __device__ inline int act_stride(int n) { return pad32(n) + 2; }  // == 2 (mod 32)

// one layer: acc = in[BM x K] @ W^T[K x N]; TPW = column tiles per wave, G = k-steps per group
template <int RS, int TPW, int MAXT, int NW>
LGX_DEV void mlp_layer(const float* __restrict__ in_lds, int s_in, const float* __restrict__ W, int K, int N,
                       int wave, int ln16, int lq, f32x4 (&acc)[RS][MAXT]) {
  constexpr int G = 8 / TPW;
  const int Kp = pad32(K);
  int col[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) col[t] = min((wave + NW * t) * 16 + ln16, N - 1);
  float bA[G][TPW], bB[G][TPW];
  // Every lane loads, from a clamped row / column of W, with no select: padding columns
  // (col >= N) only feed accumulator columns the epilogue discards, and rows k >= K meet the
  // zero-padded activation columns (finite weights x 0 = 0).  A conditional load or select here
  // compiles to an exec-masked branch or an early vmcnt wait per load, serialising the B stream.
  // 32-bit byte offsets from the SGPR base.
  const char* Wb = reinterpret_cast<const char*>(W);
  auto load = [&](float (&b)[G][TPW], int k0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t row = (uint32_t)(min(k0 + 4 * g + lq, K - 1) * N);
#pragma unroll
      for (int t = 0; t < TPW; ++t) b[g][t] = *reinterpret_cast<const float*>(Wb + (row + (uint32_t)col[t]) * 4u);
    }
  };
  // A fragments (activations in LDS) are read one group ahead as well, so the MFMAs of a group
  // never wait on their own LDS read
  float aA[G][RS], aB[G][RS];
  auto loadA = [&](float (&av)[G][RS], int k0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int r = 0; r < RS; ++r) av[g][r] = in_lds[(r * 16 + ln16) * s_in + k0 + 4 * g + lq];
  };
  auto compute = [&](const float (&b)[G][TPW], const float (&av)[G][RS]) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int r = 0; r < RS; ++r)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][r], b[g][t], acc[r][t], 0, 0, 0);
  };
  constexpr int KG = 4 * G;  // k per group
  load(bA, 0);
  loadA(aA, 0);
  for (int k0 = 0; k0 < Kp; k0 += 2 * KG) {
    if (k0 + KG < Kp) { load(bB, k0 + KG); loadA(aB, k0 + KG); }
    compute(bA, aA);
    if (k0 + KG >= Kp) break;
    if (k0 + 2 * KG < Kp) { load(bA, k0 + 2 * KG); loadA(aA, k0 + 2 * KG); }
    compute(bB, aB);
  }
}

template <int RS, int ACTW, int MAXT, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_num_vgpr(LGX_MLP_MAX_VGPR)))
lgx_mlp_forward_kernel(MlpBatch batch) {
  constexpr int NT = 64 * NW;
  constexpr int BM = 16 * RS;
  __shared__ float act_lds[BM * ACTW];
  const MlpArgs& a = batch.m[blockIdx.y];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ln16 = lane & 15;
  const int lq = lane >> 4;
  const int64_t ntiles_rows = (a.rows + BM - 1) / BM;

  for (int64_t tile = blockIdx.x; tile < ntiles_rows; tile += gridDim.x) {
    const int64_t r0 = tile * BM;
    const int K0 = a.dims[0];
    const int K0p = pad32(K0);
    int s_in = act_stride(K0);
    int in_off = 0;
    for (int idx = tid; idx < BM * K0p; idx += NT) {
      int r = idx / K0p, k = idx - r * K0p;
      int64_t gr = r0 + r;
      act_lds[r * s_in + k] = (gr < a.rows && k < K0) ? a.x[gr * K0 + k] : 0.f;
    }
    __syncthreads();
    for (int l = 0; l < a.nl; ++l) {
      const int K = a.dims[l], N = a.dims[l + 1];
      const bool last = l == a.nl - 1;
      const int s_out = act_stride(N);
      const int out_off = (in_off == 0) ? ACTW * BM - BM * s_out : 0;
      const int ntile = pad16(N) >> 4;
      const int tpw = (ntile + NW - 1) / NW;
      f32x4 acc[RS][MAXT];
#pragma unroll
      for (int r = 0; r < RS; ++r)
#pragma unroll
        for (int t = 0; t < MAXT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* in_lds = act_lds + in_off;
      if constexpr (MAXT >= 8) {
        if (tpw > 4) mlp_layer<RS, 8, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
        else if (tpw > 2) mlp_layer<RS, 4, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
        else if (tpw > 1) mlp_layer<RS, 2, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
        else mlp_layer<RS, 1, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
      } else {
        if (tpw > 1) mlp_layer<RS, 2, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
        else mlp_layer<RS, 1, MAXT, NW>(in_lds, s_in, a.wt[l], K, N, wave, ln16, lq, acc);
      }
      // epilogue: bias + activation -> LDS output region (zero pad to pad32) or Y
      const int Np32 = pad32(N);
#pragma unroll
      for (int t = 0; t < MAXT; ++t) {
        const int ct = wave + NW * t;
        if (t >= tpw) break;
        const int col = ct * 16 + ln16;
        const bool cv = col < N;
        const float bb = cv ? a.b[l][col] : 0.f;
        const float sc = (last && a.out_scale && cv) ? a.out_scale[col] : 1.f;
#pragma unroll
        for (int r = 0; r < RS; ++r)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = r * 16 + lq * 4 + i;
            const float v = acc[r][t][i] + bb;
            if (!last) {
              if (col < Np32) act_lds[out_off + row * s_out + col] = cv ? activate(v, a.act) : 0.f;
            } else if (cv) {
              const int64_t gr = r0 + row;
              if (gr < a.rows) a.y[gr * N + col] = v * sc;
            }
          }
      }
      if (!last) {
        // columns [pad16(N), pad32(N)) have no owning tile: zero them for the next layer's k reads
        const int p16 = pad16(N);
        for (int idx = tid; idx < BM * (Np32 - p16); idx += NT) {
          int r = idx / (Np32 - p16), cc = p16 + idx % (Np32 - p16);
          act_lds[out_off + r * s_out + cc] = 0.f;
        }
      }
      __syncthreads();  // outputs visible to every wave; input region free for reuse
      in_off = out_off;
      s_in = s_out;
    }
  }
}

static bool valid(const MlpArgs& a, int actw) {
  if (a.nl < 1 || a.nl > MLP_MAX_LAYERS || a.rows < 0) return false;
  for (int l = 0; l <= a.nl; ++l)
    if (a.dims[l] <= 0 || a.dims[l] > MLP_MAX_W) return false;
  for (int l = 0; l < a.nl; ++l)
    if (act_stride(a.dims[l]) + act_stride(a.dims[l + 1]) > actw) return false;
  return true;
}

static int needed_actw(const MlpArgs& a) {
  int w = 0;
  for (int l = 0; l < a.nl; ++l) {
    int s = act_stride(a.dims[l]) + act_stride(a.dims[l + 1]);
    w = s > w ? s : w;
  }
  return w;
}


static int launch_batch(const MlpBatch& b, int count, hipStream_t stream) {
  int64_t rows = 0;
  int actw = 0;
  for (int i = 0; i < count; ++i) {
    const MlpArgs& a = b.m[i];
    if (a.nl < 1 || a.nl > MLP_MAX_LAYERS) return -1;
    for (int l = 0; l <= a.nl; ++l)
      if (a.dims[l] <= 0 || a.dims[l] > MLP_MAX_W) return -1;
    rows = a.rows > rows ? a.rows : rows;
    int w = needed_actw(a);
    actw = w > actw ? w : actw;
  }
  if (rows == 0) return 0;
  int maxw = 0;
  for (int i = 0; i < count; ++i)
    for (int l = 1; l <= b.m[i].nl; ++l) maxw = b.m[i].dims[l] > maxw ? b.m[i].dims[l] : maxw;
  const bool narrow = actw <= 264 && maxw <= 128;
  if (!narrow && actw > 1032) return -1;
  // narrow nets (actuator MLP, <= 128 wide): 32-row tiles, 33 KB LDS; wide (policy): 16-row tiles
  const int bm = narrow ? 32 : 16;
  int64_t tiles = (rows + bm - 1) / bm;
  int64_t grid = tiles < 2048 ? tiles : 2048;
  dim3 g((unsigned)grid, (unsigned)count);
  if (narrow)
    LGX_LAUNCH((lgx_mlp_forward_kernel<2, 264, 2, 4>), g, dim3(256), 0, stream, b);
  else if (actw <= 776)   // 16-row tiles x 8 waves
    LGX_LAUNCH((lgx_mlp_forward_kernel<1, 776, 8, 8>), g, dim3(512), 0, stream, b);
  else
    LGX_LAUNCH((lgx_mlp_forward_kernel<1, 1032, 8, 4>), g, dim3(256), 0, stream, b);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

static void fill(MlpArgs& a, const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims,
                 const float* const* weights, const float* const* biases, int32_t act) {
  a.x = x; a.y = y; a.rows = rows; a.nl = nl; a.act = act; a.out_scale = nullptr;
  for (int l = 0; l <= nl && l <= MLP_MAX_LAYERS; ++l) a.dims[l] = dims[l];
  for (int l = 0; l < nl && l < MLP_MAX_LAYERS; ++l) { a.wt[l] = weights[l]; a.b[l] = biases[l]; }
}

int lgx_launch_mlp_forward(const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims,
                           const float* const* weights, const float* const* biases, int32_t act, hipStream_t stream) {
  if (nl < 1 || nl > MLP_MAX_LAYERS) return -1;
  MlpBatch b{};
  fill(b.m[0], x, y, rows, nl, dims, weights, biases, act);
  return launch_batch(b, 1, stream);
}

int lgx_launch_mlp_forward2(const lgx_mlp_desc* d, int32_t count, hipStream_t stream) {
  if (count < 1 || count > 2) return -1;
  MlpBatch b{};
  for (int i = 0; i < count; ++i) {
    if (d[i].nl < 1 || d[i].nl > MLP_MAX_LAYERS) return -1;
    fill(b.m[i], d[i].x, d[i].y, d[i].rows, d[i].nl, d[i].dims, d[i].weights, d[i].biases, d[i].act);
  }
  return launch_batch(b, count, stream);
}

#include "lgx_actuator_ws.h"

__global__ void __launch_bounds__(256, 2) lgx_actuator_ws_kernel(WsArgs a) { actuator_ws_body(a, blockIdx.x, gridDim.x); }

// packed actuator weights: W0t[30x128] b0 W1t[128x128] b1 W2t[128x128] b2 W3t[128x3] b3 (see lgx.h):
// the weight-stationary f32-MFMA body (lgx_actuator_ws.h), the one the post-physics launch runs
int lgx_launch_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale,
                            hipStream_t stream, int wg_per_cu) {
  if (rows <= 0) return 0;
  WsArgs wa{in, out, rows, w, out_scale};
  const int64_t tiles = (rows + WS_BM - 1) / WS_BM;
  const int grid = (int)std::min<int64_t>(tiles, 256 * std::max(1, wg_per_cu));
  LGX_LAUNCH(lgx_actuator_ws_kernel, dim3(grid), dim3(256), 0, stream, wa);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------- ANYmal SEA LSTM
// One thread per joint row: 2-layer LSTM(2->8) + Linear(8->1) (anymal.py:62-78).  Tiny
// (~1.1 kFLOP per joint); weights read through the scalar cache.
__global__ void lgx_lstm_kernel(const float* __restrict__ x, float* __restrict__ h, float* __restrict__ c,
                                float* __restrict__ tau, int64_t m, const float* __restrict__ w) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  const float* in_s = w;
  const float* out_s = w + 2;
  const float* p = w + 3;
  const float* Wih0 = p; p += 64;
  const float* Whh0 = p; p += 256;
  const float* bih0 = p; p += 32;
  const float* bhh0 = p; p += 32;
  const float* Wih1 = p; p += 256;
  const float* Whh1 = p; p += 256;
  const float* bih1 = p; p += 32;
  const float* bhh1 = p; p += 32;
  const float* Wl = p;
  const float* bl = p + 8;
  float inp[8];
  inp[0] = x[r * 2] * in_s[0];
  inp[1] = x[r * 2 + 1] * in_s[1];
#pragma unroll
  for (int L = 0; L < 2; ++L) {
    const float* Wih = L ? Wih1 : Wih0;
    const float* Whh = L ? Whh1 : Whh0;
    const float* bih = L ? bih1 : bih0;
    const float* bhh = L ? bhh1 : bhh0;
    const int ni = L ? 8 : 2;
    float* hh = h + ((int64_t)L * m + r) * 8;
    float* cc = c + ((int64_t)L * m + r) * 8;
    float hv[8], cv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { hv[k] = hh[k]; cv[k] = cc[k]; }
    float g[32];
#pragma unroll
    for (int gi = 0; gi < 32; ++gi) {
      float s = bih[gi] + bhh[gi];
      for (int i = 0; i < ni; ++i) s += Wih[gi * ni + i] * inp[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) s += Whh[gi * 8 + i] * hv[i];
      g[gi] = s;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float ig = 1.f / (1.f + expf(-g[k])), fg = 1.f / (1.f + expf(-g[8 + k]));
      float gg = tanhf(g[16 + k]), og = 1.f / (1.f + expf(-g[24 + k]));
      cv[k] = fg * cv[k] + ig * gg;
      hv[k] = og * tanhf(cv[k]);
      cc[k] = cv[k];
      hh[k] = hv[k];
      inp[k] = hv[k];
    }
  }
  float s = bl[0];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += Wl[i] * inp[i];
  tau[r] = out_s[0] * s;
}

int lgx_launch_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w,
                             hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(lgx_lstm_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, x, h, c, tau, m, w);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
