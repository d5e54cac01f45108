// PPO-side kernels.  GAE (rsl_rl RolloutStorage.compute_returns): the reference issues ~6
// elementwise launches per step of the T-step backward recursion; here one thread owns one
// env and walks the T steps backwards in registers (coalesced [T,N] rows per step).
#include "lgx_device.h"
#include "lgx_internal.h"

#include <algorithm>

// Chan et al.'s pairwise combination of (count, mean, M2) summaries (M2 = sum of squared
// deviations from the mean): no cancellation when |mean| >> std, unlike sum / sum-of-squares
struct MomentSummary {
  double n, mean, m2;
};
LGX_DEV MomentSummary moments_combine(MomentSummary a, MomentSummary b) {
  const double n = a.n + b.n;
  if (n == 0.0) return a;
  const double d = b.mean - a.mean;
  return {n, a.mean + d * (b.n / n), a.m2 + b.m2 + d * d * (a.n * b.n / n)};
}

// part != nullptr: each workgroup also writes the (count, mean, M2) of its advantages (double,
// Welford per thread over its T steps, then a fixed-order Chan tree) to part[3 * blockIdx.x ...]
// for lgx_adv_norm_kernel
__global__ void __launch_bounds__(256) lgx_gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                      const uint8_t* __restrict__ dones,
                                                      const float* __restrict__ last_val, float* __restrict__ ret,
                                                      float* __restrict__ adv, int32_t T, int32_t N, float gamma,
                                                      float lam, double* __restrict__ part) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  MomentSummary ms = {0.0, 0.0, 0.0};
  if (e < N) {
    float next_v = last_val[e];
    float a = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      int64_t i = (int64_t)t * N + e;
      float v = val[i];
      float nt = 1.0f - (float)dones[i];
      float delta = rew[i] + nt * gamma * next_v - v;
      a = delta + nt * gamma * lam * a;
      float r = a + v;
      ret[i] = r;
      const float d = r - v;
      adv[i] = d;
      ms.n += 1.0;                       // Welford
      const double dd = (double)d - ms.mean;
      ms.mean += dd / ms.n;
      ms.m2 += dd * ((double)d - ms.mean);
      next_v = v;
    }
  }
  if (!part) return;
  __shared__ MomentSummary rs[256];
  rs[threadIdx.x] = ms;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) rs[threadIdx.x] = moments_combine(rs[threadIdx.x], rs[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = rs[0].n;
    part[3 * blockIdx.x + 1] = rs[0].mean;
    part[3 * blockIdx.x + 2] = rs[0].m2;
  }
}

// rsl_rl's advantage normalisation, (adv - adv.mean()) / (adv.std() + 1e-8) with the unbiased
// std, in place: every workgroup re-combines the GAE summaries in the same order (double), then
// normalises its slice in f32 as torch does from the f32 mean / std.  The summaries may cover more
// samples than the n normalised here (data-parallel: every rank's summaries, in rank order)
__global__ void __launch_bounds__(256) lgx_adv_norm_kernel(float* __restrict__ adv, int64_t n,
                                                           const double* __restrict__ part, int32_t nparts) {
  __shared__ float ms[2];
  if (threadIdx.x == 0) {
    MomentSummary s = {0.0, 0.0, 0.0};
    for (int i = 0; i < nparts; ++i) s = moments_combine(s, {part[3 * i], part[3 * i + 1], part[3 * i + 2]});
    const double var = s.n > 1.0 ? s.m2 / (s.n - 1.0) : 0.0;
    ms[0] = (float)s.mean;
    ms[1] = (float)sqrt(var) + 1e-8f;
  }
  __syncthreads();
  const float mean = ms[0], den = ms[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adv[i] = (adv[i] - mean) / den;
}

int lgx_launch_gae(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                   float* adv, int32_t T, int32_t N, float gamma, float lam, hipStream_t stream) {
  if (T <= 0 || N <= 0) return -1;
  hipLaunchKernelGGL(lgx_gae_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, rew, val, dones, last_val, ret, adv, T,
                     N, gamma, lam, (double*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_gae_parts(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                         float* adv, int32_t T, int32_t N, float gamma, float lam, double* parts, hipStream_t stream) {
  if (T <= 0 || N <= 0) return -1;
  hipLaunchKernelGGL(lgx_gae_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, rew, val, dones, last_val, ret, adv, T,
                     N, gamma, lam, parts);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_adv_norm(float* adv, int64_t n, const double* parts, int32_t nparts, hipStream_t stream) {
  if (n <= 0 || nparts <= 0) return -1;
  const int blocks = (int)std::min<int64_t>((n + 1023) / 1024, 256);
  hipLaunchKernelGGL(lgx_adv_norm_kernel, dim3(blocks), dim3(256), 0, stream, adv, n, parts, nparts);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_gae_norm(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                        float* adv, int32_t T, int32_t N, float gamma, float lam, double* scratch, hipStream_t stream) {
  if (T <= 0 || N <= 0) return -1;
  const int nparts = (N + 255) / 256;
  hipLaunchKernelGGL(lgx_gae_kernel, dim3(nparts), dim3(256), 0, stream, rew, val, dones, last_val, ret, adv, T, N,
                     gamma, lam, scratch);
  const int64_t n = (int64_t)T * N;
  const int blocks = (int)std::min<int64_t>((n + 1023) / 1024, 256);
  hipLaunchKernelGGL(lgx_adv_norm_kernel, dim3(blocks), dim3(256), 0, stream, adv, n, (const double*)scratch, nparts);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
