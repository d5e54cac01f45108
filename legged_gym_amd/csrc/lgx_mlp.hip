// Fused MLP forward on f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32, one rounding per product,
// the f32 matrix peak of gfx950).  Used for
//   * the Go1 actuator network (UniNet core, go1.py:22-35,100-105): 30-128-128-128-3, tanh,
//     evaluated for decimation x N x 4 leg rows per env-step in ONE launch (the reference runs
//     4 legs x 4 substeps of small GEMMs plus 96 host<->device copies per env-step);
//   * rsl_rl ActorCritic inference in the rollout (obs-512-256-128-{12,1}, ELU).
//
// Tiling: a 256-thread workgroup (4 waves) owns BM = 32 rows for ALL layers; the activation
// tile stays in LDS between layers (ping-pong, padded row stride -> conflict-free column
// reads), so HBM traffic = input rows + output rows + weights (L2-resident).  Each wave owns
// output column tiles w, w+4, ... (32 columns each, <= 4 per wave for widths <= 512);
// A fragments come from LDS (lane l: row l&31, k = k0 + (l>>5)), B fragments from the
// transposed weights W^T [in][out] in global memory (lane l: column l&31 -> coalesced 128 B).
#include "lgx_device.h"
#include "lgx_internal.h"

#define MLP_BM 32
#define MLP_THREADS 256
#define MLP_MAX_W 512
#define MLP_LDS_STRIDE (MLP_MAX_W + 4)
#define MLP_MAX_LAYERS 6

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct MlpArgs {
  int32_t nl;
  int32_t dims[MLP_MAX_LAYERS + 1];
  const float* wt[MLP_MAX_LAYERS];  // [in][out]
  const float* b[MLP_MAX_LAYERS];
  int32_t act;                      // 1 elu, 2 tanh
  const float* out_scale;           // optional per-output-column scale
};

LGX_DEV float activate(float x, int act) {
  if (act == 1) return x > 0.f ? x : expm1f(x);
  if (act == 2) return tanhf(x);
  return x;
}

__global__ void __launch_bounds__(MLP_THREADS)
lgx_mlp_forward_kernel(const float* __restrict__ X, float* __restrict__ Y, int64_t rows, MlpArgs a) {
  __shared__ float lds[2 * MLP_BM * MLP_LDS_STRIDE];  // 132 KB static (gfx950: 160 KB LDS per CU)
  float* buf0 = lds;
  float* buf1 = lds + MLP_BM * MLP_LDS_STRIDE;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * MLP_BM;
  const int k0 = a.dims[0];
  const int k0p = (k0 + 1) & ~1;
  // stage input tile (zero-padded rows and the odd K column)
  for (int idx = tid; idx < MLP_BM * k0p; idx += MLP_THREADS) {
    int r = idx / k0p, k = idx - r * k0p;
    int64_t gr = r0 + r;
    buf0[r * MLP_LDS_STRIDE + k] = (gr < rows && k < k0) ? X[gr * k0 + k] : 0.f;
  }
  __syncthreads();
  float* in = buf0;
  float* out = buf1;
  const int arow = lane & 31;
  const int akk = lane >> 5;
  for (int l = 0; l < a.nl; ++l) {
    const int K = a.dims[l], Nn = a.dims[l + 1];
    const int Kp = (K + 1) & ~1;
    const int ntiles = (Nn + 31) >> 5;
    const float* __restrict__ W = a.wt[l];
    const float* __restrict__ bias = a.b[l];
    const bool last = l == a.nl - 1;
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    int col[4];
    bool cv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      int tile = wave + 4 * t;
      col[t] = tile * 32 + arow;
      cv[t] = tile < ntiles && col[t] < Nn;
    }
    const bool any = wave < ntiles;
    if (any) {
      for (int k = 0; k < Kp; k += 2) {
        int kk = k + akk;
        float av = in[arow * MLP_LDS_STRIDE + kk];
        bool kval = kk < K;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (wave + 4 * t < ntiles) {  // wave-uniform
            float bv = (cv[t] && kval) ? W[(int64_t)kk * Nn + col[t]] : 0.f;
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
          }
        }
      }
    }
    // epilogue: bias + activation -> next LDS tile or Y
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      int tile = wave + 4 * t;
      if (tile >= ntiles) continue;
      int c = tile * 32 + (lane & 31);
      if (c >= Nn) continue;
      float bb = bias[c];
      float sc = (last && a.out_scale) ? a.out_scale[c] : 1.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        int r = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        float v = acc[t][i] + bb;
        if (!last) {
          out[r * MLP_LDS_STRIDE + c] = activate(v, a.act);
        } else {
          int64_t gr = r0 + r;
          if (gr < rows) Y[gr * Nn + c] = v * sc;
        }
      }
    }
    if (!last) {
      // zero the odd pad column used by the next layer's k-pairs
      if ((Nn & 1) && tid < MLP_BM) out[tid * MLP_LDS_STRIDE + Nn] = 0.f;
      __syncthreads();
      float* t = in; in = out; out = t;
    }
  }
}

static int launch_mlp(const float* x, float* y, int64_t rows, const MlpArgs& a, hipStream_t stream) {
  if (rows <= 0) return 0;
  for (int l = 0; l <= a.nl; ++l)
    if (a.dims[l] <= 0 || a.dims[l] > MLP_MAX_W) return -1;
  int64_t blocks = (rows + MLP_BM - 1) / MLP_BM;
  hipLaunchKernelGGL(lgx_mlp_forward_kernel, dim3((unsigned)blocks), dim3(MLP_THREADS), 0, stream, x, y, rows, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_mlp_forward(const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims,
                           const float* const* weights, const float* const* biases, int32_t act, hipStream_t stream) {
  if (nl < 1 || nl > MLP_MAX_LAYERS) return -1;
  MlpArgs a{};
  a.nl = nl;
  for (int l = 0; l <= nl; ++l) a.dims[l] = dims[l];
  for (int l = 0; l < nl; ++l) { a.wt[l] = weights[l]; a.b[l] = biases[l]; }
  a.act = act;
  a.out_scale = nullptr;
  return launch_mlp(x, y, rows, a, stream);
}

// packed actuator weights: W0t[30x128] b0 W1t[128x128] b1 W2t[128x128] b2 W3t[128x3] b3 (see lgx.h)
int lgx_launch_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale,
                            hipStream_t stream) {
  MlpArgs a{};
  a.nl = 4;
  const int d[5] = {30, 128, 128, 128, 3};
  const float* p = w;
  for (int l = 0; l < 4; ++l) {
    a.dims[l] = d[l];
    a.wt[l] = p; p += d[l] * d[l + 1];
    a.b[l] = p; p += d[l + 1];
  }
  a.dims[4] = 3;
  a.act = 2;
  a.out_scale = out_scale;
  return launch_mlp(in, out, rows, a, stream);
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
