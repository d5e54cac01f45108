// PPO-side kernels.  GAE (rsl_rl RolloutStorage.compute_returns): the reference issues ~6
// elementwise launches per step of the T-step backward recursion; here one thread owns one
// env and walks the T steps backwards in registers (coalesced [T,N] rows per step).
#include "lgx_device.h"
#include "lgx_internal.h"

__global__ void lgx_gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                               const uint8_t* __restrict__ dones, const float* __restrict__ last_val,
                               float* __restrict__ ret, float* __restrict__ adv, int32_t T, int32_t N, float gamma,
                               float lam) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
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
    adv[i] = r - v;
    next_v = v;
  }
}

int lgx_launch_gae(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                   float* adv, int32_t T, int32_t N, float gamma, float lam, hipStream_t stream) {
  if (T <= 0 || N <= 0) return -1;
  hipLaunchKernelGGL(lgx_gae_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, rew, val, dones, last_val, ret, adv, T,
                     N, gamma, lam);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
