// lgx PPO update kernels: everything of one rsl_rl PPO minibatch step (rsl_rl v1.0.x
// `PPO.update`, configured by legged_robot_config.py:226-239) that is not a GEMM:
//   - minibatch row gather,
//   - bias + ELU epilogue of the actor/critic hidden layers (net-major [2, M, H] activations),
//   - the PPO loss and its analytic gradient w.r.t. the action mean, value and std
//     (clipped surrogate, clipped value loss, entropy bonus; Normal(mu, std) log-prob), with
//     the KL used by the adaptive learning-rate schedule,
//   - output-layer backward (dZ3 = (dMU W4) * elu'(A3), dW4, db3 partials),
//   - ELU backward fused with the bias-gradient column sums,
//   - split-K / per-chunk partial reductions straight into the flat gradient buffer,
//   - global-norm gradient clipping (clip_grad_norm_) fused into the Adam step.
// The GEMMs between them are the hand-written split-bf16 kernels (lgx_gemm_x3p.hip forwards and
// dA, lgx_gemm_tn.hip dW; lgx_gemm_split.hip / lgx_gemm.hip variants), with library GEMMs through
// torch only for shapes they do not take or LGX_PPO_GEMM=lib (rl/fused_ppo.py).  All reductions are
// two-stage in a fixed order (bitwise reproducible); the adaptive learning rate and the Adam
// step counter live on the device so a whole update can be captured in one hipGraph.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>


#include "lgx_internal.h"

namespace {

constexpr int TPB = 256;
constexpr int CHUNK = 64;  // rows per workgroup in the backward epilogues
constexpr int HEAD_CHUNK = 32;  // rows per workgroup in the output-layer backward
constexpr int LOSS_TPB = 64;    // rows per loss workgroup (384 workgroups per 24576-row minibatch)

__device__ __forceinline__ float elu_f(float x) { return lgx_elu(x); }
__device__ __forceinline__ float elu_grad_from_out(float y) { return y > 0.f ? 1.f : y + 1.f; }

// rsl_rl adaptive schedule (PPO.update): lr /= 1.5 if KL > 2 kl*, *= 1.5 if 0 < KL < kl*/2,
// bounded [1e-5, 1e-2]; python-float (double) arithmetic as upstream
__device__ __forceinline__ void adapt_lr(double kl, double* lr, double desired_kl) {
  double l = lr[0];
  if (kl > desired_kl * 2.0) l = fmax(1e-5, l / 1.5);
  else if (desired_kl / 2.0 > kl && kl > 0.0) l = fmin(1e-2, l * 1.5);
  lr[0] = l;
}

// ---------------------------------------------------------------------------------------- gather
__global__ void __launch_bounds__(TPB)
gather_rows_kernel(const float* __restrict__ src, float* __restrict__ dst, const int64_t* __restrict__ idx,
                   int64_t rows, int32_t width) {
  // one row per 64-lane wave, 4 rows per workgroup
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* s = src + idx[r] * width;
  float* d = dst + r * width;
  for (int c = lane; c < width; c += 64) d[c] = s[c];
}

// ---------------------------------------------------------------------------------------- rollout
// PPO.act + RolloutStorage.add_transitions for one env step (rsl_rl v1.0.x): actions =
// mu + std * eps (Normal.sample with the caller's standard-normal draws), log-prob, and the
// storage row t (obs, critic obs, actions, value, log-prob, mu, sigma).  16 envs per workgroup
// (256 workgroups at 4096 envs): the obs rows of those envs are one contiguous range, copied
// with 16-byte accesses when aligned.
constexpr int ACT_ENVS = 16;

__device__ __forceinline__ void copy_rows(const float* __restrict__ src, float* __restrict__ dst, int64_t cnt) {
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t c4 = cnt >> 2;
    for (int64_t i = threadIdx.x; i < c4; i += TPB)
      reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
    for (int64_t i = 4 * c4 + threadIdx.x; i < cnt; i += TPB) dst[i] = src[i];
  } else {
    for (int64_t i = threadIdx.x; i < cnt; i += TPB) dst[i] = src[i];
  }
}
// STORE: also the previous step's lgx_ppo_store rows (env n0 + threadIdx.x), which read only that
// step's env outputs and storage row: one launch per env step instead of two
template <bool STORE>
__global__ void __launch_bounds__(TPB)
ppo_act_kernel(lgx_ppo_act_args a, lgx_ppo_store_args ps) {
  const int64_t n0 = (int64_t)blockIdx.x * ACT_ENVS;
  const int64_t nn = min((int64_t)ACT_ENVS, a.num_envs - n0);
  if (STORE && threadIdx.x < nn) {
    const int64_t n = n0 + threadIdx.x;
    ps.st_rew[n] = ps.time_outs ? lgx_ppo_reward(ps.rew[n], ps.gamma, ps.st_values[n], ps.time_outs[n] != 0) : ps.rew[n];
    ps.st_dones[n] = ps.reset[n] ? 1 : 0;
  }
  copy_rows(a.obs + n0 * a.num_obs, a.st_obs + n0 * a.num_obs, nn * a.num_obs);
  if (a.cobs && a.st_cobs) copy_rows(a.cobs + n0 * a.num_cobs, a.st_cobs + n0 * a.num_cobs, nn * a.num_cobs);
  const int A = a.num_actions;
  for (int64_t k = threadIdx.x; k < nn * A; k += TPB) {  // coalesced [env, action] elements
    const int64_t e = n0 * A + k;
    const int j = (int)(k % A);
    const float sd = a.std[j];
    const float mu = a.mu[e];
    const float act = lgx_ppo_sample(mu, sd, a.noise[e]);
    a.actions_out[e] = act;
    a.st_actions[e] = act;
    a.st_mu[e] = mu;
    a.st_sigma[e] = sd;
  }
  __syncthreads();
  if (threadIdx.x < nn) {
    const int64_t n = n0 + threadIdx.x;
    float logp = 0.f;
    for (int j = 0; j < A; ++j) logp += lgx_ppo_logp_term(a.st_actions[n * A + j] - a.mu[n * A + j], a.std[j]);
    a.st_logp[n] = logp;
    if (a.value) a.st_values[n] = a.value[n];
  }
}

// PPO.process_env_step: r += gamma * V * time_out (time-out bootstrap), dones stored as bytes
__global__ void __launch_bounds__(TPB)
ppo_store_kernel(lgx_ppo_store_args a) {
  const int64_t n = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (n >= a.num_envs) return;
  a.st_rew[n] = a.time_outs ? lgx_ppo_reward(a.rew[n], a.gamma, a.st_values[n], a.time_outs[n] != 0) : a.rew[n];
  a.st_dones[n] = a.reset[n] ? 1 : 0;
}

// ---------------------------------------------------------------------------------------- bias + act
__global__ void __launch_bounds__(TPB)
bias_act_kernel(float* __restrict__ z, const float* __restrict__ b, int64_t rows, int32_t cols, int32_t nets,
                int32_t act) {
  const int64_t per_net = rows * cols;
  const int64_t n4 = per_net * nets / 4;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n4; i += (int64_t)gridDim.x * TPB) {
    int64_t e = i * 4;
    int net = (int)(e / per_net);
    int c = (int)(e % cols);
    float4 v = reinterpret_cast<float4*>(z)[i];
    const float* bb = b + net * cols + c;
    v.x += bb[0]; v.y += bb[1]; v.z += bb[2]; v.w += bb[3];
    if (act == 1) { v.x = elu_f(v.x); v.y = elu_f(v.y); v.z = elu_f(v.z); v.w = elu_f(v.w); }
    else if (act == 2) { v.x = tanhf(v.x); v.y = tanhf(v.y); v.z = tanhf(v.z); v.w = tanhf(v.w); }
    reinterpret_cast<float4*>(z)[i] = v;
  }
}

// ---------------------------------------------------------------------------------------- loss
// One row per thread.  Partials per workgroup (row sums, fixed-order tree-free reduction):
//   [0, A)      d loss / d std_j          (log-prob path; the entropy term is added in finalize)
//   [A, 2A)     d loss / d b4a_j          (= sum of dMU over rows)
//   2A          d loss / d b4c            (= sum of dV)
//   2A+1        KL sum, 2A+2 surrogate sum, 2A+3 value-loss sum
// HEAD: the output layers are computed here too (mu_raw = A3a W4a^T, v_raw = A3c w4c^T from the
// last hidden activations, instead of two library GEMMs): 256 threads per 64 rows, 4 lanes per
// row each dot a quarter of the H columns (16-byte loads, weights broadcast from LDS), combined
// across the 4 lanes in a fixed order; then one thread per row as without HEAD.
template <bool HEAD>
__global__ void __launch_bounds__(HEAD ? 4 * LOSS_TPB : LOSS_TPB)
ppo_loss_kernel(lgx_ppo_loss_args a) {
  constexpr int MAXA = LGX_PPO_MAX_ACTIONS;
  const int A = a.num_actions;
  const int NP = 2 * A + 4;
  __shared__ float red[LOSS_TPB][2 * MAXA + 4 + 1];
  __shared__ float hout[HEAD ? LOSS_TPB : 1][MAXA + 1];
  if constexpr (HEAD) {
    extern __shared__ float4 wsh[];               // [A + 1][H / 4]: W4a rows, then w4c
    const int H = a.hidden, H4 = H >> 2;
    for (int i = threadIdx.x; i < (A + 1) * H4; i += 4 * LOSS_TPB)
      wsh[i] = i < A * H4 ? reinterpret_cast<const float4*>(a.W4a)[i]
                          : reinterpret_cast<const float4*>(a.W4c)[i - A * H4];
    __syncthreads();
    const int lr = threadIdx.x >> 2, q = threadIdx.x & 3;
    const int64_t row = min((int64_t)blockIdx.x * LOSS_TPB + lr, a.rows - 1);   // clamped: tail rows unused
    const int qn = H4 >> 2;                       // float4 columns per lane
    const float4* xa = reinterpret_cast<const float4*>(a.head_in + row * H) + q * qn;
    const float4* xc = reinterpret_cast<const float4*>(a.head_in + (a.rows + row) * H) + q * qn;
    float acc[MAXA + 1];
#pragma unroll
    for (int j = 0; j <= MAXA; ++j) acc[j] = 0.f;
    for (int c = 0; c < qn; ++c) {
      const float4 x = xa[c], y = xc[c];
      const int col = q * qn + c;
#pragma unroll
      for (int j = 0; j < MAXA; ++j) {
        if (j < A) {
          const float4 w = wsh[j * H4 + col];
          acc[j] += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
        }
      }
      const float4 w = wsh[A * H4 + col];
      acc[MAXA] += y.x * w.x + y.y * w.y + y.z * w.z + y.w * w.w;
    }
#pragma unroll
    for (int j = 0; j <= MAXA; ++j) {             // lanes q = 0..3 of a row are adjacent
      float v = acc[j];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      acc[j] = v;
    }
    if (q == 0) {
#pragma unroll
      for (int j = 0; j < MAXA; ++j)
        if (j < A) hout[lr][j] = acc[j];
      hout[lr][MAXA] = acc[MAXA];
    }
    __syncthreads();
    if (threadIdx.x >= LOSS_TPB) {                // rows are handled by the first 64 threads
      __syncthreads();
      return;
    }
  }
  const int64_t r = (int64_t)blockIdx.x * LOSS_TPB + threadIdx.x;
  float* my = red[threadIdx.x];
  for (int k = 0; k < NP; ++k) my[k] = 0.f;
  if (r < a.rows) {
    const int64_t g = a.idx ? a.idx[r] : r;
    const float invM = 1.0f / (float)a.rows;
    float mu[MAXA], sd[MAXA], act[MAXA];
    float logp = 0.f, kl = 0.f;
    const float half_log_2pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
    for (int j = 0; j < A; ++j) {
      mu[j] = (HEAD ? hout[threadIdx.x][j] : a.mu_raw[r * A + j]) + a.b4a[j];
      sd[j] = a.std[j];
      act[j] = a.actions[g * A + j];
      float var = sd[j] * sd[j];
      float d = act[j] - mu[j];
      logp += -(d * d) / (2.f * var) - logf(sd[j]) - half_log_2pi;
      float so = a.old_sigma[g * A + j], mo = a.old_mu[g * A + j];
      kl += logf(sd[j] / so + 1.e-5f) + (so * so + (mo - mu[j]) * (mo - mu[j])) / (2.f * var) - 0.5f;
    }
    const float adv = a.advantages[g];
    const float ratio = expf(logp - a.old_logp[g]);
    const float lo = 1.f - a.clip_param, hi = 1.f + a.clip_param;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float s1 = -adv * ratio, s2 = -adv * rc;
    const bool inside = ratio >= lo && ratio <= hi;
    // torch.maximum backward: ties split the gradient; clamp passes it inside [lo, hi]
    float dsdr;
    if (s1 > s2) dsdr = -adv;
    else if (s1 < s2) dsdr = inside ? -adv : 0.f;
    else dsdr = 0.5f * (-adv) + 0.5f * (inside ? -adv : 0.f);
    const float surr = fmaxf(s1, s2);
    const float dlogp = dsdr * invM * ratio;
    for (int j = 0; j < A; ++j) {
      float var = sd[j] * sd[j];
      float d = act[j] - mu[j];
      float dm = dlogp * d / var;
      a.d_mu[r * A + j] = dm;
      my[A + j] = dm;
      my[j] = dlogp * (d * d / (var * sd[j]) - 1.f / sd[j]);
    }
    // value loss
    const float v = (HEAD ? hout[threadIdx.x][MAXA] : a.v_raw[r]) + a.b4c[0];
    const float tv = a.target_values[g], ret = a.returns[g];
    float vl, dv;
    if (a.use_clipped_value_loss) {
      float dvt = v - tv;
      float vc = tv + fminf(fmaxf(dvt, -a.clip_param), a.clip_param);
      bool vin = dvt >= -a.clip_param && dvt <= a.clip_param;
      float u1 = (v - ret) * (v - ret), u2 = (vc - ret) * (vc - ret);
      vl = fmaxf(u1, u2);
      float g1 = 2.f * (v - ret), g2 = vin ? 2.f * (vc - ret) : 0.f;
      dv = u1 > u2 ? g1 : (u1 < u2 ? g2 : 0.5f * g1 + 0.5f * g2);
    } else {
      vl = (ret - v) * (ret - v);
      dv = 2.f * (v - ret);
    }
    dv *= a.value_loss_coef * invM;
    a.d_v[r] = dv;
    my[2 * A] = dv;
    my[2 * A + 1] = kl;
    my[2 * A + 2] = surr;
    my[2 * A + 3] = vl;
  }
  __syncthreads();
  if (threadIdx.x < NP) {
    float s = 0.f;
    for (int t = 0; t < LOSS_TPB; ++t) s += red[t][threadIdx.x];
    a.partials[(int64_t)blockIdx.x * NP + threadIdx.x] = s;
  }
}

// one workgroup: reduce the loss partials, write d std / d b4a / d b4c into the flat gradient,
// the KL mean and the running loss sums.  Thread (g, k): value k over partial blocks g, g+8, ...
// then a fixed-order combine of the 8 groups.
// 64-lane sum in a fixed butterfly order (every lane of the wave gets it)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// sq (optional): the sum of squares of the gradient entries written here (d std, d b4a, d b4c) ->
// *sq, and the optimizer step counter advanced (the clip norm's partial for
// lgx_adam_clip_mirror_sq; lgx_reduce_slices_sq)
__device__ void loss_finalize(const lgx_ppo_loss_args& a, int32_t nblocks, float* sq = nullptr,
                              int64_t* step = nullptr) {   // TPB threads
  const int A = a.num_actions;
  const int NP = 2 * A + 4;               // <= 36
  __shared__ float red[8][2 * LGX_PPO_MAX_ACTIONS + 4];
  const int grp = threadIdx.x / 32;
  {
    for (int kk = threadIdx.x % 32; kk < NP; kk += 32) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;   // 4 independent chains, fixed order
      int b = grp;
      for (; b + 24 < nblocks; b += 32) {
        s0 += a.partials[(int64_t)b * NP + kk];
        s1 += a.partials[(int64_t)(b + 8) * NP + kk];
        s2 += a.partials[(int64_t)(b + 16) * NP + kk];
        s3 += a.partials[(int64_t)(b + 24) * NP + kk];
      }
      for (; b < nblocks; b += 8) s0 += a.partials[(int64_t)b * NP + kk];
      red[grp][kk] = (s0 + s1) + (s2 + s3);
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (sq && t < 64) {   // wave 0 (NP <= 36 lanes hold values): squares of the written entries
    float v = 0.f;
    if (t < NP) {
      float s2 = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) s2 += red[g][t];
      v = t < A ? s2 - a.entropy_coef / a.std[t] : t <= 2 * A ? s2 : 0.f;
    }
    v = wave_sum(v * v);
    if (t == 0) {
      *sq = v;
      if (step) step[0] += 1;
    }
  }
  if (t >= NP) return;
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) s += red[g][t];
  const float invM = 1.0f / (float)a.rows;
  if (t < A) a.g_std[t] = s - a.entropy_coef / a.std[t];   // entropy: -c_e mean(sum_j log std_j + c)
  else if (t < 2 * A) a.g_b4a[t - A] = s;
  else if (t == 2 * A) a.g_b4c[0] = s;
  else if (t == 2 * A + 1) {
    const float kl = s * invM;
    a.stats[0] = kl;                                         // KL mean of this minibatch (local)
    if (a.lr) adapt_lr((double)kl, a.lr, a.desired_kl);     // single process: schedule applied here
  }
  else if (t == 2 * A + 2) a.stats[1] += s * invM;         // running surrogate-loss sum
  else a.stats[2] += s * invM;                             // running value-loss sum
}

__global__ void __launch_bounds__(TPB)
ppo_loss_finalize_kernel(lgx_ppo_loss_args a, int32_t nblocks) { loss_finalize(a, nblocks); }

__global__ void adapt_lr_kernel(const float* __restrict__ kl_sum, float kl_scale, double* __restrict__ lr,
                                double desired_kl) {
  adapt_lr((double)(kl_sum[0] * kl_scale), lr, desired_kl);
}

// ---------------------------------------------------------------------------------------- head bwd
// per 32-row chunk: dW4 partial = [dMU | dV]^T [A3a | A3c], dZ3 = (dMU W4a | dV w4c) * elu'(A3)
// written over A3, db3 partial = column sums of dZ3.  Partials row: [A*H (dW4a), H (dW4c), 2H (db3)].
// Thread = (net, column c): one coalesced pass over the chunk's rows keeps the head-weight column
// and the dW4 column accumulators in registers; dMU rows are LDS broadcasts.
template <int MAXA>
__global__ void __launch_bounds__(TPB)
head_bwd_kernel(const float* __restrict__ d_mu, const float* __restrict__ d_v, const float* __restrict__ W4a,
                const float* __restrict__ W4c, float* __restrict__ A3, int64_t rows, int32_t A, int32_t H,
                float* __restrict__ partials, lgx_ppo_loss_args fin, int32_t fin_blocks) {
  // fin_blocks > 0: one extra (last) workgroup runs the loss finalize (it reads only the loss
  // partials, complete at launch), so the finalize costs no launch of its own
  if (fin_blocks > 0 && blockIdx.x == gridDim.x - 1) {
    loss_finalize(fin, fin_blocks);
    return;
  }
  constexpr int DS = ((MAXA + 1 + 3) / 4) * 4;  // dMU row (+ dV) padded for 16-byte LDS reads
  __shared__ __align__(16) float dmu[HEAD_CHUNK][DS];
  const int64_t r0 = (int64_t)blockIdx.x * HEAD_CHUNK;
  const int nr = (int)min((int64_t)HEAD_CHUNK, rows - r0);
  for (int i = threadIdx.x; i < HEAD_CHUNK * (A + 1); i += TPB) {
    int rr = i / (A + 1), j = i % (A + 1);
    float v = 0.f;
    if (rr < nr) v = j < A ? d_mu[(r0 + rr) * A + j] : d_v[r0 + rr];
    dmu[rr][j] = v;
  }
  __syncthreads();
  float* P = partials + (int64_t)blockIdx.x * ((A + 1) * H + 2 * H);
  for (int o = threadIdx.x; o < 2 * H; o += TPB) {
    const int net = o / H, c = o % H;
    float w[MAXA], acc[MAXA];
    const int nj = net == 0 ? A : 1;
#pragma unroll
    for (int j = 0; j < MAXA; ++j) {
      w[j] = j < nj ? (net == 0 ? W4a[j * H + c] : W4c[c]) : 0.f;
      acc[j] = 0.f;
    }
    const int jo = net == 0 ? 0 : A;  // dMU column block of this net
    float* col = A3 + (int64_t)net * rows * H + r0 * H + c;
    float cs = 0.f;
    for (int rr = 0; rr < nr; ++rr) {
      float y = col[(int64_t)rr * H];
      float drow[DS];
#pragma unroll
      for (int q = 0; q < DS / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(&dmu[rr][4 * q]);
        drow[4 * q] = v.x; drow[4 * q + 1] = v.y; drow[4 * q + 2] = v.z; drow[4 * q + 3] = v.w;
      }
      float dA = 0.f;
      if (net == 0) {
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
          if (j < nj) { acc[j] += drow[j] * y; dA += drow[j] * w[j]; }
      } else {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j <= MAXA; ++j) d = (j == A) ? drow[j] : d;   // dV column
        acc[0] += d * y;
        dA = d * w[0];
      }
      float dz = dA * elu_grad_from_out(y);
      col[(int64_t)rr * H] = dz;
      cs += dz;
    }
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
      if (j < nj) P[(jo + j) * H + c] = acc[j];
    P[(A + 1) * H + o] = cs;
  }
}

// ---------------------------------------------------------------------------------------- loss + head bwd
// lgx_ppo_loss_bwd: ppo_loss_kernel<true> and head_bwd_kernel of LB_ROWS rows per workgroup in
// ONE launch.  The rows' last hidden activations of both networks are read from HBM once into LDS
// (row stride H + 4 floats), then
//   1. output layers: LB_LPR lanes per row dot interleaved float4 columns against the head
//      weights (LDS broadcasts), combined across the row's lanes by xor shuffles;
//   2. loss and its gradient per row: the row's lanes take actions j = q, q + LB_LPR, ...
//      (log-prob / KL partials combined by shuffles), dMU / dV into LDS, loss partials per
//      workgroup (fixed-order row sums, same layout as ppo_loss_kernel's);
//   3. output-layer backward (thread = (net, column)): dZ3 = (dMU W4a | dV w4c) * elu'(A3) over
//      head_in in place, dW4 and db3 partials per workgroup (head_bwd_kernel's layout).
// The loss finalize (d std, head-bias gradients, KL, stats, adaptive LR) runs later on one extra
// workgroup of lgx_reduce_slices_finalize (it needs every workgroup's partials).
#ifndef LGX_LB_ROWS
#define LGX_LB_ROWS 32
#endif
constexpr int LB_ROWS = LGX_LB_ROWS;   // rows per workgroup (16 or 32: TPB / LB_ROWS lanes per row)
static_assert(LB_ROWS == 16 || LB_ROWS == 32, "lanes per row must divide a wave");
constexpr int LB_LPR = TPB / LB_ROWS;   // lanes per row in phases 1-2 (8)

__device__ __forceinline__ float lb_rowsum(float v) {   // sum over the LB_LPR lanes of a row
#pragma unroll
  for (int m = 1; m < LB_LPR; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

template <int MAXA>
__global__ void __launch_bounds__(TPB)
ppo_loss_bwd_kernel(lgx_ppo_loss_args a, float* __restrict__ hparts) {
  constexpr int JQ = (MAXA + LB_LPR - 1) / LB_LPR;   // actions per lane
  constexpr int DS = ((MAXA + 1 + 3) / 4) * 4;      // dMU row (+ dV), 16-byte LDS reads
  const int A = a.num_actions, H = a.hidden, H4 = H >> 2, HS = H + 4;
  const int NP = 2 * A + 4;
  extern __shared__ float4 lb_dyn[];
  float* ylds = reinterpret_cast<float*>(lb_dyn);            // [2][LB_ROWS][HS]
  float* wlds = ylds + 2 * LB_ROWS * HS;                      // [A + 1][H]: W4a rows, then w4c
  __shared__ __align__(16) float dmu[LB_ROWS][DS];
  __shared__ float red[LB_ROWS][2 * MAXA + 4 + 1];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * LB_ROWS;
  const int nr = (int)min((int64_t)LB_ROWS, a.rows - r0);
  float* A3 = const_cast<float*>(a.head_in);
  // ---- stage the rows (rows past M as zeros) and the head weights
  for (int i = t; i < 2 * LB_ROWS * H4; i += TPB) {
    const int nrow = i / H4, c4 = i - nrow * H4;              // nrow = net * LB_ROWS + row
    const int net = nrow >= LB_ROWS, rr = nrow - net * LB_ROWS;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rr < nr) v = reinterpret_cast<const float4*>(A3 + ((int64_t)net * a.rows + r0 + rr) * H)[c4];
    *reinterpret_cast<float4*>(ylds + nrow * HS + 4 * c4) = v;
  }
  for (int i = t; i < (A + 1) * H4; i += TPB)
    reinterpret_cast<float4*>(wlds)[i] = i < A * H4 ? reinterpret_cast<const float4*>(a.W4a)[i]
                                                    : reinterpret_cast<const float4*>(a.W4c)[i - A * H4];
  __syncthreads();
  // ---- 1. output layers
  const int rr = t / LB_LPR, q = t % LB_LPR;
  float hv[MAXA + 1];
#pragma unroll
  for (int j = 0; j <= MAXA; ++j) hv[j] = 0.f;
  {
    const float* ya = ylds + rr * HS;
    const float* yc = ylds + (LB_ROWS + rr) * HS;
    const float4* w4 = reinterpret_cast<const float4*>(wlds);
    for (int c4 = q; c4 < H4; c4 += LB_LPR) {
      const float4 x = *reinterpret_cast<const float4*>(ya + 4 * c4);
      const float4 y = *reinterpret_cast<const float4*>(yc + 4 * c4);
#pragma unroll
      for (int j = 0; j < MAXA; ++j)
        if (j < A) {
          const float4 w = w4[j * H4 + c4];
          hv[j] += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
        }
      const float4 w = w4[A * H4 + c4];
      hv[MAXA] += y.x * w.x + y.y * w.y + y.z * w.z + y.w * w.w;
    }
  }
#pragma unroll
  for (int j = 0; j <= MAXA; ++j) hv[j] = lb_rowsum(hv[j]);
  // ---- 2. loss per row (lane q: actions q + LB_LPR m)
  float* my = red[rr];
  const bool valid = rr < nr;
  {
    const int64_t r = r0 + rr;
    const int64_t g = valid ? (a.idx ? a.idx[r] : r) : 0;
    const float invM = 1.0f / (float)a.rows;
    const float half_log_2pi = 0.91893853320467274178f;
    float mu[JQ], sd[JQ], act[JQ];
    float logp = 0.f, kl = 0.f;
#pragma unroll
    for (int m = 0; m < JQ; ++m) {
      const int j = q + LB_LPR * m;
      float h = 0.f;
#pragma unroll
      for (int jj = 0; jj < MAXA; ++jj) h = jj == j ? hv[jj] : h;
      mu[m] = sd[m] = 1.f;
      act[m] = 0.f;
      if (valid && j < A) {
        mu[m] = h + a.b4a[j];
        sd[m] = a.std[j];
        act[m] = a.actions[g * A + j];
        const float var = sd[m] * sd[m];
        const float d = act[m] - mu[m];
        logp += -(d * d) / (2.f * var) - logf(sd[m]) - half_log_2pi;
        const float so = a.old_sigma[g * A + j], mo = a.old_mu[g * A + j];
        kl += logf(sd[m] / so + 1.e-5f) + (so * so + (mo - mu[m]) * (mo - mu[m])) / (2.f * var) - 0.5f;
      }
    }
    logp = lb_rowsum(logp);
    kl = lb_rowsum(kl);
    float dlogp = 0.f, surr = 0.f, vl = 0.f, dv = 0.f;
    if (valid) {
      const float adv = a.advantages[g];
      const float ratio = expf(logp - a.old_logp[g]);
      const float lo = 1.f - a.clip_param, hi = 1.f + a.clip_param;
      const float rc = fminf(fmaxf(ratio, lo), hi);
      const float s1 = -adv * ratio, s2 = -adv * rc;
      const bool inside = ratio >= lo && ratio <= hi;
      float dsdr;   // torch.maximum backward: ties split the gradient; clamp passes it inside [lo, hi]
      if (s1 > s2) dsdr = -adv;
      else if (s1 < s2) dsdr = inside ? -adv : 0.f;
      else dsdr = 0.5f * (-adv) + 0.5f * (inside ? -adv : 0.f);
      surr = fmaxf(s1, s2);
      dlogp = dsdr * invM * ratio;
      const float v = hv[MAXA] + a.b4c[0];
      const float tv = a.target_values[g], ret = a.returns[g];
      if (a.use_clipped_value_loss) {
        const float dvt = v - tv;
        const float vc = tv + fminf(fmaxf(dvt, -a.clip_param), a.clip_param);
        const bool vin = dvt >= -a.clip_param && dvt <= a.clip_param;
        const float u1 = (v - ret) * (v - ret), u2 = (vc - ret) * (vc - ret);
        vl = fmaxf(u1, u2);
        const float g1 = 2.f * (v - ret), g2 = vin ? 2.f * (vc - ret) : 0.f;
        dv = u1 > u2 ? g1 : (u1 < u2 ? g2 : 0.5f * g1 + 0.5f * g2);
      } else {
        vl = (ret - v) * (ret - v);
        dv = 2.f * (v - ret);
      }
      dv *= a.value_loss_coef * invM;
    }
#pragma unroll
    for (int m = 0; m < JQ; ++m) {
      const int j = q + LB_LPR * m;
      if (j < A) {
        const float var = sd[m] * sd[m];
        const float d = act[m] - mu[m];
        const float dm = valid ? dlogp * d / var : 0.f;
        dmu[rr][j] = dm;
        my[A + j] = dm;
        my[j] = valid ? dlogp * (d * d / (var * sd[m]) - 1.f / sd[m]) : 0.f;
      }
    }
    if (q == 0) {
      dmu[rr][A] = dv;
      my[2 * A] = dv;
      my[2 * A + 1] = valid ? kl : 0.f;
      my[2 * A + 2] = surr;
      my[2 * A + 3] = vl;
    }
  }
  __syncthreads();
  if (t < NP) {   // loss partials of this workgroup (rows in order)
    float s = 0.f;
    for (int i = 0; i < LB_ROWS; ++i) s += red[i][t];
    a.partials[(int64_t)blockIdx.x * NP + t] = s;
  }
  // ---- 3. output-layer backward (as head_bwd_kernel; A3 rows from LDS)
  float* P = hparts + (int64_t)blockIdx.x * ((A + 1) * H + 2 * H);
  for (int o = t; o < 2 * H; o += TPB) {
    const int net = o >= H, c = o - net * H;
    const int nj = net == 0 ? A : 1;
    float w[MAXA], acc[MAXA];
#pragma unroll
    for (int j = 0; j < MAXA; ++j) {
      w[j] = j < nj ? wlds[(net == 0 ? j : A) * H + c] : 0.f;
      acc[j] = 0.f;
    }
    const float* ycol = ylds + net * LB_ROWS * HS + c;
    float* col = A3 + ((int64_t)net * a.rows + r0) * H + c;
    float cs = 0.f;
    for (int i = 0; i < nr; ++i) {
      const float y = ycol[i * HS];
      float drow[DS];
#pragma unroll
      for (int u = 0; u < DS / 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(&dmu[i][4 * u]);
        drow[4 * u] = v.x; drow[4 * u + 1] = v.y; drow[4 * u + 2] = v.z; drow[4 * u + 3] = v.w;
      }
      float dA = 0.f;
      if (net == 0) {
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
          if (j < nj) { acc[j] += drow[j] * y; dA += drow[j] * w[j]; }
      } else {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j <= MAXA; ++j) d = (j == A) ? drow[j] : d;   // dV column
        acc[0] += d * y;
        dA = d * w[0];
      }
      const float dz = dA * elu_grad_from_out(y);
      col[(int64_t)i * H] = dz;
      cs += dz;
    }
    const int jo = net == 0 ? 0 : A;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
      if (j < nj) P[(jo + j) * H + c] = acc[j];
    P[(A + 1) * H + o] = cs;
  }
}

// ---------------------------------------------------------------------------------------- elu bwd
// dA [nets, rows, H] -> dZ = dA * elu'(Y) in place; partial column sums per 64-row chunk:
// partials[chunk][net*H + c].  Thread = 4 consecutive columns (16-B loads and stores).
__global__ void __launch_bounds__(TPB)
elu_bwd_colsum_kernel(float* __restrict__ dA, const float* __restrict__ Y, int64_t rows, int32_t H, int32_t nets,
                      float* __restrict__ partials) {
  const int net = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * CHUNK;
  const int nr = (int)min((int64_t)CHUNK, rows - r0);
  const int64_t base = (int64_t)net * rows * H + r0 * H;
  float* P = partials + (int64_t)blockIdx.x * nets * H + net * H;
  const int H4 = H >> 2;
  // TPB threads = (row lane, column quad): rows are split over TPB / H4 lanes; widths whose H4
  // does not divide TPB leave the last TPB % H4 threads idle, widths above TPB walk the column
  // quads in uniform rounds (every thread reaches every barrier)
  const int lanes_per_row = H4 < TPB ? H4 : TPB;
  const int row_groups = TPB / lanes_per_row;
  const int cq = threadIdx.x % lanes_per_row, rg = threadIdx.x / lanes_per_row;
  __shared__ float4 red[TPB];
  for (int c0 = 0; c0 < H4; c0 += lanes_per_row) {
    const int c4 = c0 + cq;
    const bool active = c4 < H4 && rg < row_groups;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
      for (int rr = rg; rr < nr; rr += row_groups) {
        int64_t i = (base + (int64_t)rr * H) / 4 + c4;
        float4 d = reinterpret_cast<float4*>(dA)[i];
        float4 y = reinterpret_cast<const float4*>(Y)[i];
        d.x *= elu_grad_from_out(y.x); d.y *= elu_grad_from_out(y.y);
        d.z *= elu_grad_from_out(y.z); d.w *= elu_grad_from_out(y.w);
        reinterpret_cast<float4*>(dA)[i] = d;
        cs.x += d.x; cs.y += d.y; cs.z += d.z; cs.w += d.w;
      }
    }
    red[threadIdx.x] = cs;
    __syncthreads();
    if (rg == 0 && c4 < H4) {
      float4 t = red[cq];
      for (int g = 1; g < row_groups; ++g) {
        float4 u = red[g * lanes_per_row + cq];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      reinterpret_cast<float4*>(P)[c4] = t;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------- reductions
// job: dst[j][i] = sum_s src[j*job_stride + s*slice_stride + i] for s < S, i < n, j < count.
// Workgroup = one tile of OT outputs of one job; its 256 / OT lane groups split the slices
// (s = g, g + 256/OT, ...) and combine in LDS in a fixed order.  OT = 64 for short slice loops
// (split-K partials, 8 slices), 16 for long ones (per-chunk bias / head partials, hundreds of
// slices): independent loads in flight instead of one serial chain per output.
// Jobs whose offsets, strides and n are multiples of 4 floats (16-byte aligned: the split-K weight
// partials) run on float4 lanes (tile_outputs < 0: -4 x 64 outputs per workgroup, 64 lanes x 4
// slice groups), the rest on scalar lanes.
// One reduction tile b; returns this lane's sum of squares of the outputs it wrote (wave 0's lanes
// write).  Ends with a barrier (the LDS scratch is reused by the workgroup's next tile).
__device__ __forceinline__ float reduce_tile(const lgx_reduce_jobs& jobs, int32_t njobs, int b, float* red,
                                             float4* red4) {
  int ji = 0;
  while (ji + 1 < njobs && b >= jobs.tile_start[ji + 1]) ++ji;
  const lgx_reduce_job& jb = jobs.job[ji];
  const int ot = jobs.tile_outputs[ji];
  float q2 = 0.f;
  if (ot < 0) {   // float4 path: 64 lanes x 4 outputs per group, TPB / 64 groups over the slices
    const int groups = TPB / 64;
    const int t = threadIdx.x, oi = t % 64, g = t / 64;
    const int64_t o4 = (int64_t)(b - jobs.tile_start[ji]) * 64 + oi;   // float4 output index
    const int64_t total4 = (int64_t)jb.count * jb.n / 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t j = 0, i = 0;
    if (o4 < total4) {
      j = (4 * o4) / jb.n;
      i = 4 * o4 - j * jb.n;
      const float* s = jb.src + j * jb.job_stride + i;
#pragma unroll 8
      for (int k = g; k < jb.slices; k += groups) {
        const float4 v = *reinterpret_cast<const float4*>(s + (int64_t)k * jb.slice_stride);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    red4[t] = acc;
    __syncthreads();
    if (g == 0 && o4 < total4) {
      float4 sum = red4[oi];
      for (int q = 1; q < groups; ++q) {
        const float4 u = red4[q * 64 + oi];
        sum.x += u.x; sum.y += u.y; sum.z += u.z; sum.w += u.w;
      }
      *reinterpret_cast<float4*>(jb.dst + j * jb.dst_stride + i) = sum;
      q2 = sum.x * sum.x + sum.y * sum.y + sum.z * sum.z + sum.w * sum.w;
    }
  } else {
    const int groups = TPB / ot;
    const int t = threadIdx.x, oi = t % ot, g = t / ot;
    const int64_t o = (int64_t)(b - jobs.tile_start[ji]) * ot + oi;
    const int64_t total = (int64_t)jb.count * jb.n;
    float acc = 0.f;
    int64_t j = 0, i = 0;
    if (o < total) {
      j = o / jb.n;
      i = o % jb.n;
      const float* s = jb.src + j * jb.job_stride + i;
#pragma unroll 8
      for (int k = g; k < jb.slices; k += groups) acc += s[(int64_t)k * jb.slice_stride];
    }
    red[t] = acc;
    __syncthreads();
    if (g == 0 && o < total) {   // (the g == 0 lanes t < ot <= 64 are in wave 0)
      float sum = red[oi];
      for (int q = 1; q < groups; ++q) sum += red[q * ot + oi];
      jb.dst[j * jb.dst_stride + i] = sum;
      q2 = sum * sum;
    }
  }
  __syncthreads();
  return q2;
}

// Persistent over the tiles (workgroup w: tiles w, w + nwg, ...).  sq (optional): sq[workgroup] =
// the sum of squares of every output it wrote (fixed order: tiles in order per lane, then wave 0's
// lanes by butterfly), so the clip norm needs no pass of its own over the gradient
__global__ void __launch_bounds__(TPB)
reduce_slices_kernel(lgx_reduce_jobs jobs, int32_t njobs, int32_t ntiles, lgx_ppo_loss_args fin, int32_t fin_blocks,
                     float* sq, int64_t* step) {
  // workgroup 0: the deferred loss finalize of lgx_ppo_loss_bwd (first, so its serial partial
  // sums overlap the reduction tiles instead of trailing them)
  if (fin_blocks > 0 && blockIdx.x == 0) {
    loss_finalize(fin, fin_blocks, sq, step);
    return;
  }
  __shared__ float red[TPB];
  __shared__ float4 red4[TPB];
  const int f = fin_blocks > 0 ? 1 : 0;
  const int nwg = (int)gridDim.x - f;
  float q2 = 0.f;
  for (int b = (int)blockIdx.x - f; b < ntiles; b += nwg) q2 += reduce_tile(jobs, njobs, b, red, red4);
  if (sq && threadIdx.x < 64) {
    q2 = wave_sum(q2);
    if (threadIdx.x == 0) sq[blockIdx.x] = q2;
  }
}

// ---------------------------------------------------------------------------------------- clip + Adam
// stage 1: per-block sums of squares of (scale * g); block 0 also advances the step counter
__global__ void __launch_bounds__(TPB)
sumsq_kernel(const float* __restrict__ g, int64_t n, float scale, float* __restrict__ partials,
             int64_t* __restrict__ step) {
  __shared__ float red[TPB];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    float v = g[i] * scale;
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = TPB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = red[0];
    if (blockIdx.x == 0 && step) step[0] += 1;
  }
}

// stage 2: every block re-reduces the (few) partials -> global norm -> clip coefficient
// (torch clip_grad_norm_: coef = min(max_norm / (norm + 1e-6), 1)), then torch Adam
// (fused form: step_size = lr / bc1; denom = sqrt(v) / sqrt(bc2) + eps)
// Mirrors: derived copies of parameter blocks that the next minibatch's GEMMs read (zero-padded
// layer-1 weights, transposed hidden weights; lgx_copy2d job layout with src inside p) written
// with the updated value, so no weight-preparation pass runs between minibatches.
// round-to-nearest-even bf16 (as v_cvt_pk_bf16_f32, finite inputs)
__device__ __forceinline__ uint16_t bf16_rne(float x) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float fx2_t __attribute__((ext_vector_type(2)));
  return (uint16_t)__builtin_bit_cast(uint32_t, __builtin_convertvector((fx2_t){x, 0.f}, bf16x2_t));
}

struct Mirror {
  int64_t off, dst_ld, dst_bs;  // off: first flat index of the block in p
  float* dst;
  int32_t count, rows, cols, transpose;   // count = batch * rows * cols
  uint64_t inv_rc, inv_cols;    // ceil(2^40 / (rows * cols)), ceil(2^40 / cols): exact quotients
};                              // for every index < count (host-checked: count * rows * cols < 2^40)

// floor(l / d) for l < 2^20-ish ranges as one 64-bit multiply-shift (inv = ceil(2^40 / d), exact
// while l * d < 2^40) instead of the ~40-instruction 32-bit integer division, three per element
__device__ __forceinline__ int32_t mdiv(int32_t l, uint64_t inv) { return (int32_t)(((uint64_t)l * inv) >> 40); }
constexpr int MAX_MIRRORS = LGX_MAX_REDUCE_JOBS;
struct Mirrors {
  Mirror mj[MAX_MIRRORS];
  int32_t n;
};

// one mirror element: updated parameter value pi at (batch b, row rr, col cc) of block J
__device__ __forceinline__ void mirror_store(const Mirror& J, int32_t b, int32_t rr, int32_t cc, float pi) {
  if (J.transpose & 2) {   // bf16 limb layout of lgx_split_bf16 (split-bf16 GEMM operand)
    const int32_t nn = (J.transpose & 1) ? cc : rr, kk = (J.transpose & 1) ? rr : cc;
    const int32_t kout = (J.transpose & 1) ? J.rows : J.cols;
    uint16_t* d = reinterpret_cast<uint16_t*>(J.dst) + b * J.dst_bs + x3_limb_off(nn, kk, 0, (kout + 31) >> 5);
    const uint16_t l0 = bf16_rne(pi);
    const float r1 = pi - __uint_as_float((uint32_t)l0 << 16);
    const uint16_t l1 = bf16_rne(r1);
    d[0] = l0;                   // limb l at + l * 128 * 32
    d[4096] = l1;
    d[8192] = bf16_rne(r1 - __uint_as_float((uint32_t)l1 << 16));
  } else {
    J.dst[b * J.dst_bs + (J.transpose ? (int64_t)cc * J.dst_ld + rr : (int64_t)rr * J.dst_ld + cc)] = pi;
  }
}

// One parameter per thread (consecutive lanes: consecutive elements, so a non-transposed limb
// mirror's 2-byte stores coalesce); the clip coefficient and the bias corrections (double pow)
// computed once per workgroup.
__global__ void __launch_bounds__(TPB)
adam_clip_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v, int64_t n,
                 const float* __restrict__ partials, int32_t nparts, float grad_scale, float max_norm,
                 const double* __restrict__ lr, const int64_t* __restrict__ step, float beta1, float beta2, float eps,
                 Mirrors mir) {
  __shared__ float red[TPB];
  __shared__ float coef_s, step_size_s, bc2_sqrt_s;
  // this thread's first AE elements loaded before the prologue: their HBM latency overlaps the
  // partial-sum reduction and the bias corrections instead of following them (clamped addresses)
  constexpr int AE = 3;
  const int64_t stride = (int64_t)gridDim.x * TPB, i0 = (int64_t)blockIdx.x * TPB + threadIdx.x;
  float pp[AE], gg[AE], mm[AE], vv[AE];
#pragma unroll
  for (int u = 0; u < AE; ++u) {
    const int64_t i = min(i0 + u * stride, n - 1);
    pp[u] = p[i]; gg[u] = g[i]; mm[u] = m[i]; vv[u] = v[i];
  }
  float s = 0.f;
  {   // (lgx_adam_clip_mirror_sq reads up to ~1k partials: 16-byte loads)
    const int n4 = ((uintptr_t)partials & 15) == 0 ? nparts / 4 : 0;
    for (int i = threadIdx.x; i < n4; i += TPB) {
      const float4 v = reinterpret_cast<const float4*>(partials)[i];
      s += (v.x + v.y) + (v.z + v.w);
    }
    for (int i = 4 * n4 + threadIdx.x; i < nparts; i += TPB) s += partials[i];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = TPB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0]);
    const float c = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    coef_s = fminf(c, 1.f) * grad_scale;
    const double t = (double)step[0];
    const float bc1 = (float)(1.0 - pow((double)beta1, t));
    const float bc2 = (float)(1.0 - pow((double)beta2, t));
    step_size_s = (float)(lr[0] / (double)bc1);
    bc2_sqrt_s = sqrtf(bc2);
  }
  __syncthreads();
  const float coef = coef_s, step_size = step_size_s, bc2_sqrt = bc2_sqrt_s;
  auto update = [&](int64_t i, float p0, float g0, float m0, float v0) {
    const float gi = g0 * coef;
    g[i] = gi;
    const float mi = beta1 * m0 + (1.f - beta1) * gi;
    const float vi = beta2 * v0 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    const float pi = p0 - step_size * mi / denom;
    p[i] = pi;
    for (int q = 0; q < mir.n; ++q) {
      const Mirror& J = mir.mj[q];
      const uint64_t li = (uint64_t)(i - J.off);
      if (li < (uint64_t)J.count) {
        const int32_t l = (int32_t)li, rc = J.rows * J.cols;
        const int32_t b = mdiv(l, J.inv_rc), rem = l - b * rc, rr = mdiv(rem, J.inv_cols), cc = rem - rr * J.cols;
        mirror_store(J, b, rr, cc, pi);
      }
    }
  };
#pragma unroll
  for (int u = 0; u < AE; ++u)
    if (i0 + u * stride < n) update(i0 + u * stride, pp[u], gg[u], mm[u], vv[u]);
  for (int64_t i = i0 + AE * stride; i < n; i += stride) update(i, p[i], g[i], m[i], v[i]);
}

}  // namespace

// ---------------------------------------------------------------------------------------- C-ABI
#define LGX_STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" int lgx_ppo_gather_rows(const float* src, float* dst, const int64_t* idx, int64_t rows, int32_t width,
                                   void* stream) {
  if (!src || !dst || !idx || rows < 0 || width <= 0) return lgx_fail(LGX_EINVAL, "lgx_ppo_gather_rows: bad args");
  if (rows == 0) return LGX_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(TPB), 0, LGX_STREAM(stream), src, dst,
                     idx, rows, width);
  return lgx_hip_status("lgx_ppo_gather_rows");
}

static bool act_args_ok(const lgx_ppo_act_args& a) {
  return !(a.num_envs <= 0 || a.num_actions <= 0 || a.num_obs <= 0 || !a.mu || !a.std || !a.noise || !a.obs ||
           !a.actions_out || !a.st_obs || !a.st_actions || (a.value && !a.st_values) || !a.st_logp || !a.st_mu ||
           !a.st_sigma || ((a.cobs != nullptr) != (a.st_cobs != nullptr)));
}
static bool store_args_ok(const lgx_ppo_store_args& a) {
  return !(a.num_envs <= 0 || !a.rew || !a.reset || !a.st_values || !a.st_rew || !a.st_dones);
}

extern "C" int lgx_ppo_act(const lgx_ppo_act_args* args, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_ppo_act: null args");
  const lgx_ppo_act_args& a = *args;
  if (!act_args_ok(a)) return lgx_fail(LGX_EINVAL, "lgx_ppo_act: bad args");
  hipLaunchKernelGGL(ppo_act_kernel<false>, dim3((unsigned)((a.num_envs + ACT_ENVS - 1) / ACT_ENVS)), dim3(TPB), 0,
                     LGX_STREAM(stream), a, lgx_ppo_store_args{});
  return lgx_hip_status("lgx_ppo_act");
}

extern "C" int lgx_ppo_act_store(const lgx_ppo_act_args* args, const lgx_ppo_store_args* prev, void* stream) {
  if (!args || !prev) return lgx_fail(LGX_EINVAL, "lgx_ppo_act_store: null args");
  const lgx_ppo_act_args& a = *args;
  if (!act_args_ok(a) || !store_args_ok(*prev) || prev->num_envs != a.num_envs)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_act_store: bad args (the store must cover the same envs)");
  hipLaunchKernelGGL(ppo_act_kernel<true>, dim3((unsigned)((a.num_envs + ACT_ENVS - 1) / ACT_ENVS)), dim3(TPB), 0,
                     LGX_STREAM(stream), a, *prev);
  return lgx_hip_status("lgx_ppo_act_store");
}

extern "C" int lgx_ppo_store(const lgx_ppo_store_args* args, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_ppo_store: null args");
  const lgx_ppo_store_args& a = *args;
  if (!store_args_ok(a)) return lgx_fail(LGX_EINVAL, "lgx_ppo_store: bad args");
  hipLaunchKernelGGL(ppo_store_kernel, dim3((unsigned)((a.num_envs + TPB - 1) / TPB)), dim3(TPB), 0,
                     LGX_STREAM(stream), a);
  return lgx_hip_status("lgx_ppo_store");
}

extern "C" int lgx_bias_act(float* z, const float* b, int64_t rows, int32_t cols, int32_t nets, int32_t act,
                            void* stream) {
  if (!z || !b || rows < 0 || cols <= 0 || cols % 4 || nets <= 0 || act < 0 || act > 2)
    return lgx_fail(LGX_EINVAL, "lgx_bias_act: bad args (cols must be a multiple of 4)");
  if (rows == 0) return LGX_OK;
  int64_t n4 = rows * cols * nets / 4;
  int blocks = (int)std::min<int64_t>((n4 + TPB - 1) / TPB, 4096);
  hipLaunchKernelGGL(bias_act_kernel, dim3(blocks), dim3(TPB), 0, LGX_STREAM(stream), z, b, rows, cols, nets, act);
  return lgx_hip_status("lgx_bias_act");
}

extern "C" int64_t lgx_ppo_loss_partials_floats(int64_t rows, int32_t num_actions) {
  return ((rows + LOSS_TPB - 1) / LOSS_TPB) * (2 * (int64_t)num_actions + 4);
}

extern "C" int lgx_ppo_loss(const lgx_ppo_loss_args* args, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_ppo_loss: null args");
  lgx_ppo_loss_args a = *args;
  if (a.rows <= 0 || a.num_actions <= 0 || a.num_actions > LGX_PPO_MAX_ACTIONS || !a.b4a ||
      !a.b4c || !a.std || !a.actions || !a.old_logp || !a.old_mu || !a.old_sigma || !a.advantages ||
      !a.target_values || !a.returns || !a.d_mu || !a.d_v || !a.partials || !a.g_std || !a.g_b4a || !a.g_b4c ||
      !a.stats)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_loss: bad args");
  int blocks = (int)((a.rows + LOSS_TPB - 1) / LOSS_TPB);
  if (a.head_in) {
    const size_t lds = (size_t)(a.num_actions + 1) * a.hidden * sizeof(float);
    if (!a.W4a || !a.W4c || a.hidden <= 0 || a.hidden % 16 || lds > 65536)
      return lgx_fail(LGX_EINVAL, "lgx_ppo_loss: bad output-layer args (hidden % 16, (A+1)*hidden*4 <= 64 KB)");
    hipLaunchKernelGGL(ppo_loss_kernel<true>, dim3(blocks), dim3(4 * LOSS_TPB), lds, LGX_STREAM(stream), a);
  } else {
    if (!a.mu_raw || !a.v_raw) return lgx_fail(LGX_EINVAL, "lgx_ppo_loss: mu_raw / v_raw or head_in required");
    hipLaunchKernelGGL(ppo_loss_kernel<false>, dim3(blocks), dim3(LOSS_TPB), 0, LGX_STREAM(stream), a);
  }
  if (!a.defer_finalize)
    hipLaunchKernelGGL(ppo_loss_finalize_kernel, dim3(1), dim3(TPB), 0, LGX_STREAM(stream), a, blocks);
  return lgx_hip_status("lgx_ppo_loss");
}

extern "C" int lgx_ppo_adapt_lr(const float* kl_sum, float kl_scale, double* lr, double desired_kl, void* stream) {
  if (!kl_sum || !lr) return lgx_fail(LGX_EINVAL, "lgx_ppo_adapt_lr: bad args");
  hipLaunchKernelGGL(adapt_lr_kernel, dim3(1), dim3(1), 0, LGX_STREAM(stream), kl_sum, kl_scale, lr, desired_kl);
  return lgx_hip_status("lgx_ppo_adapt_lr");
}

extern "C" int64_t lgx_head_bwd_partials_floats(int64_t rows, int32_t num_actions, int32_t hidden) {
  return ((rows + HEAD_CHUNK - 1) / HEAD_CHUNK) * ((int64_t)(num_actions + 1) * hidden + 2 * (int64_t)hidden);
}

static int head_bwd_launch(const lgx_ppo_loss_args* fin, const float* d_mu, const float* d_v, const float* W4a,
                           const float* W4c, float* A3, int64_t rows, int32_t num_actions, int32_t hidden,
                           float* partials, void* stream) {
  if (!d_mu || !d_v || !W4a || !W4c || !A3 || !partials || rows <= 0 || num_actions <= 0 ||
      num_actions > LGX_PPO_MAX_ACTIONS || hidden <= 0 || hidden > 1024)
    return lgx_fail(LGX_EINVAL, "lgx_head_bwd: bad args");
  int blocks = (int)((rows + HEAD_CHUNK - 1) / HEAD_CHUNK);
  lgx_ppo_loss_args f{};
  int32_t fin_blocks = 0;
  if (fin) {
    f = *fin;
    fin_blocks = (int32_t)((f.rows + LOSS_TPB - 1) / LOSS_TPB);
    blocks += 1;
  }
  if (num_actions <= 12)
    hipLaunchKernelGGL(head_bwd_kernel<12>, dim3(blocks), dim3(TPB), 0, LGX_STREAM(stream), d_mu, d_v, W4a, W4c, A3,
                       rows, num_actions, hidden, partials, f, fin_blocks);
  else
    hipLaunchKernelGGL(head_bwd_kernel<LGX_PPO_MAX_ACTIONS>, dim3(blocks), dim3(TPB), 0, LGX_STREAM(stream), d_mu, d_v,
                       W4a, W4c, A3, rows, num_actions, hidden, partials, f, fin_blocks);
  return lgx_hip_status("lgx_head_bwd");
}

extern "C" int lgx_head_bwd(const float* d_mu, const float* d_v, const float* W4a, const float* W4c, float* A3,
                            int64_t rows, int32_t num_actions, int32_t hidden, float* partials, void* stream) {
  return head_bwd_launch(nullptr, d_mu, d_v, W4a, W4c, A3, rows, num_actions, hidden, partials, stream);
}

extern "C" int lgx_head_bwd_finalize(const lgx_ppo_loss_args* loss, const float* d_mu, const float* d_v,
                                     const float* W4a, const float* W4c, float* A3, int64_t rows, int32_t num_actions,
                                     int32_t hidden, float* partials, void* stream) {
  if (!loss || !loss->defer_finalize || loss->rows != rows || loss->num_actions != num_actions)
    return lgx_fail(LGX_EINVAL, "lgx_head_bwd_finalize: loss args must be the deferred-finalize lgx_ppo_loss call's");
  return head_bwd_launch(loss, d_mu, d_v, W4a, W4c, A3, rows, num_actions, hidden, partials, stream);
}

extern "C" int lgx_ppo_loss_bwd_layout(int64_t rows, int32_t num_actions, int32_t hidden, int64_t* out) {
  if (!out || rows <= 0 || num_actions <= 0 || num_actions > LGX_PPO_MAX_ACTIONS || hidden <= 0)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_loss_bwd_layout: bad args");
  const int64_t blocks = (rows + LB_ROWS - 1) / LB_ROWS;
  out[0] = blocks * (2 * (int64_t)num_actions + 4);
  out[1] = blocks * ((int64_t)(num_actions + 1) * hidden + 2 * (int64_t)hidden);
  out[2] = (int64_t)(2 * LB_ROWS * (hidden + 4) + (num_actions + 1) * hidden) * (int64_t)sizeof(float);
  return LGX_OK;
}

extern "C" int lgx_ppo_loss_bwd(const lgx_ppo_loss_args* args, float* head_partials, void* stream) {
  if (!args) return lgx_fail(LGX_EINVAL, "lgx_ppo_loss_bwd: null args");
  const lgx_ppo_loss_args& a = *args;
  if (a.rows <= 0 || a.num_actions <= 0 || a.num_actions > LGX_PPO_MAX_ACTIONS || !a.b4a || !a.b4c || !a.std ||
      !a.actions || !a.old_logp || !a.old_mu || !a.old_sigma || !a.advantages || !a.target_values || !a.returns ||
      !a.partials || !a.g_std || !a.g_b4a || !a.g_b4c || !a.stats || !head_partials)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_loss_bwd: bad args");
  if (!a.head_in || !a.W4a || !a.W4c || a.hidden <= 0 || a.hidden % 16)
    return lgx_fail(LGX_EINVAL, "lgx_ppo_loss_bwd: head_in / W4a / W4c required, hidden % 16 == 0");
  int64_t lay[3];
  lgx_ppo_loss_bwd_layout(a.rows, a.num_actions, a.hidden, lay);
  if (lay[2] > 96 * 1024) return lgx_fail(LGX_EINVAL, "lgx_ppo_loss_bwd: hidden too wide for the LDS row stage");
  static const bool attr_ok = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&ppo_loss_bwd_kernel<12>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&ppo_loss_bwd_kernel<LGX_PPO_MAX_ACTIONS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess;
  }();
  if (!attr_ok) return lgx_fail(LGX_EHIP, "lgx_ppo_loss_bwd: hipFuncSetAttribute failed");
  const int blocks = (int)((a.rows + LB_ROWS - 1) / LB_ROWS);
  // (LGX_LAUNCH on the call's last launch: a bound event, lgx_launch_bind_event, marks its end)
  if (a.defer_finalize) {
    if (a.num_actions <= 12)
      LGX_LAUNCH(ppo_loss_bwd_kernel<12>, dim3(blocks), dim3(TPB), (size_t)lay[2], LGX_STREAM(stream), a,
                 head_partials);
    else
      LGX_LAUNCH(ppo_loss_bwd_kernel<LGX_PPO_MAX_ACTIONS>, dim3(blocks), dim3(TPB), (size_t)lay[2],
                 LGX_STREAM(stream), a, head_partials);
  } else {
    if (a.num_actions <= 12)
      hipLaunchKernelGGL(ppo_loss_bwd_kernel<12>, dim3(blocks), dim3(TPB), (size_t)lay[2], LGX_STREAM(stream), a,
                         head_partials);
    else
      hipLaunchKernelGGL(ppo_loss_bwd_kernel<LGX_PPO_MAX_ACTIONS>, dim3(blocks), dim3(TPB), (size_t)lay[2],
                         LGX_STREAM(stream), a, head_partials);
    LGX_LAUNCH(ppo_loss_finalize_kernel, dim3(1), dim3(TPB), 0, LGX_STREAM(stream), a, blocks);
  }
  return lgx_hip_status("lgx_ppo_loss_bwd");
}

extern "C" int64_t lgx_colsum_partials_floats(int64_t rows, int32_t hidden, int32_t nets) {
  return ((rows + CHUNK - 1) / CHUNK) * (int64_t)hidden * nets;
}

extern "C" int lgx_elu_bwd_colsum(float* dA, const float* Y, int64_t rows, int32_t hidden, int32_t nets,
                                  float* partials, void* stream) {
  if (!dA || !Y || !partials || rows <= 0 || hidden <= 0 || hidden % 4 || nets <= 0 || nets > 2)
    return lgx_fail(LGX_EINVAL, "lgx_elu_bwd_colsum: bad args (hidden % 4)");
  int chunks = (int)((rows + CHUNK - 1) / CHUNK);
  hipLaunchKernelGGL(elu_bwd_colsum_kernel, dim3(chunks, nets), dim3(TPB), 0, LGX_STREAM(stream), dA, Y, rows, hidden,
                     nets, partials);
  return lgx_hip_status("lgx_elu_bwd_colsum");
}

constexpr int64_t LGX_REDUCE_SQ_WGS = 512;

static int reduce_slices_launch(const lgx_reduce_job* jobs, int32_t njobs, const lgx_ppo_loss_args* fin,
                                void* stream, float* sq = nullptr, int64_t* step = nullptr,
                                int64_t* blocks_out = nullptr) {
  if (!jobs || njobs <= 0 || njobs > LGX_MAX_REDUCE_JOBS) return lgx_fail(LGX_EINVAL, "lgx_reduce_slices: bad job count");
  lgx_reduce_jobs J;
  int64_t tiles = 0;
  for (int i = 0; i < njobs; ++i) {
    const lgx_reduce_job& j = jobs[i];
    if (!j.src || !j.dst || j.n <= 0 || j.slices <= 0 || j.count <= 0)
      return lgx_fail(LGX_EINVAL, "lgx_reduce_slices: bad job");
    J.job[i] = j;
    J.tile_start[i] = (int32_t)tiles;
    const bool vec = j.n % 4 == 0 && j.job_stride % 4 == 0 && j.slice_stride % 4 == 0 && j.dst_stride % 4 == 0 &&
                     ((uintptr_t)j.src & 15) == 0 && ((uintptr_t)j.dst & 15) == 0 && j.slices <= 128;
    J.tile_outputs[i] = vec ? -4 : (j.slices > 32 ? 16 : 64);
    const int64_t per = vec ? 256 : J.tile_outputs[i];
    tiles += ((int64_t)j.count * j.n + per - 1) / per;
  }
  if (tiles > (1 << 30)) return lgx_fail(LGX_EINVAL, "lgx_reduce_slices: too large");
  lgx_ppo_loss_args f{};
  int32_t fin_blocks = 0;
  if (fin) {
    f = *fin;
    fin_blocks = (int32_t)((f.rows + LB_ROWS - 1) / LB_ROWS);
    tiles += 1;
  }
  // one tile per workgroup; with sums of squares at most LGX_REDUCE_SQ_WGS persistent workgroups (the
  // partials Adam's every workgroup re-reads stay few)
  const int64_t ntiles = tiles - (fin ? 1 : 0);
  const int64_t grid = (sq || blocks_out ? std::min<int64_t>(ntiles, LGX_REDUCE_SQ_WGS) : ntiles) + (fin ? 1 : 0);
  if (blocks_out) {   // (query only: the lgx_reduce_slices_sq grid)
    *blocks_out = grid;
    return LGX_OK;
  }
  LGX_LAUNCH(reduce_slices_kernel, dim3((unsigned)grid), dim3(TPB), 0, LGX_STREAM(stream), J, njobs,
             (int32_t)ntiles, f, fin_blocks, sq, step);
  return lgx_hip_status("lgx_reduce_slices");
}

extern "C" int64_t lgx_reduce_slices_blocks(const lgx_reduce_job* jobs, int32_t njobs, int32_t with_finalize) {
  lgx_ppo_loss_args f{};
  f.rows = 1;
  int64_t n = -1;
  if (reduce_slices_launch(jobs, njobs, with_finalize ? &f : nullptr, nullptr, nullptr, nullptr, &n) != LGX_OK)
    return -1;
  return n;
}

extern "C" int lgx_reduce_slices_sq(const lgx_reduce_job* jobs, int32_t njobs, const lgx_ppo_loss_args* loss,
                                    float* sq, int64_t* step, void* stream) {
  if (!sq) return lgx_fail(LGX_EINVAL, "lgx_reduce_slices_sq: null sum-of-squares output");
  if (loss && (!loss->defer_finalize || loss->rows <= 0))
    return lgx_fail(LGX_EINVAL, "lgx_reduce_slices_sq: loss args must be a deferred-finalize lgx_ppo_loss_bwd call's");
  if (step && !loss) return lgx_fail(LGX_EINVAL, "lgx_reduce_slices_sq: the step advances on the finalize workgroup");
  return reduce_slices_launch(jobs, njobs, loss, stream, sq, step);
}

extern "C" int lgx_reduce_slices(const lgx_reduce_job* jobs, int32_t njobs, void* stream) {
  return reduce_slices_launch(jobs, njobs, nullptr, stream);
}

extern "C" int lgx_reduce_slices_finalize(const lgx_reduce_job* jobs, int32_t njobs, const lgx_ppo_loss_args* loss,
                                          void* stream) {
  if (!loss || !loss->defer_finalize || loss->rows <= 0)
    return lgx_fail(LGX_EINVAL, "lgx_reduce_slices_finalize: loss args must be a deferred-finalize lgx_ppo_loss_bwd call's");
  return reduce_slices_launch(jobs, njobs, loss, stream);
}

extern "C" int lgx_adam_clip(float* p, float* g, float* m, float* v, int64_t n, float* partials, int32_t nparts,
                             float grad_scale, float max_norm, const double* lr, int64_t* step, float beta1,
                             float beta2, float eps, void* stream) {
  if (!p || !g || !m || !v || !partials || !lr || !step || n <= 0 || nparts <= 0 || nparts > 1024)
    return lgx_fail(LGX_EINVAL, "lgx_adam_clip: bad args");
  hipLaunchKernelGGL(sumsq_kernel, dim3(nparts), dim3(TPB), 0, LGX_STREAM(stream), g, n, grad_scale, partials, step);
  int blocks = (int)std::min<int64_t>((n + TPB - 1) / TPB, 1024);
  Mirrors none{};
  hipLaunchKernelGGL(adam_clip_kernel, dim3(blocks), dim3(TPB), 0, LGX_STREAM(stream), p, g, m, v, n, partials, nparts,
                     grad_scale, max_norm, lr, step, beta1, beta2, eps, none);
  return lgx_hip_status("lgx_adam_clip");
}

static int adam_clip_mirror_launch(float* p, float* g, float* m, float* v, int64_t n, float* partials, int32_t nparts,
                                   float grad_scale, float max_norm, const double* lr, int64_t* step, float beta1,
                                   float beta2, float eps, const lgx_copy2d_job* mirrors, int32_t nmirrors,
                                   void* stream, bool presummed) {
  if (!p || !g || !m || !v || !partials || !lr || !step || n <= 0 || nparts <= 0 ||
      nparts > (presummed ? (1 << 20) : 1024) || nmirrors < 0 || nmirrors > MAX_MIRRORS || (nmirrors && !mirrors))
    return lgx_fail(LGX_EINVAL, "lgx_adam_clip_mirror: bad args");
  if (presummed && grad_scale != 1.0f)
    return lgx_fail(LGX_EINVAL, "lgx_adam_clip_mirror_sq: the presummed squares are of the unscaled gradient");
  Mirrors M{};
  M.n = nmirrors;
  for (int q = 0; q < nmirrors; ++q) {
    const lgx_copy2d_job& j = mirrors[q];
    const int64_t off = j.src - p, count = (int64_t)j.batch * j.rows * j.cols;
    // the block must be contiguous in p (src_ld == cols, src_bs == rows * cols) and inside it
    if (!j.dst || j.rows <= 0 || j.cols <= 0 || j.batch <= 0 || j.src_ld != j.cols ||
        (j.batch > 1 && j.src_bs != (int64_t)j.rows * j.cols) || off < 0 || off + count > n || count >= (1LL << 31))
      return lgx_fail(LGX_EINVAL, "lgx_adam_clip_mirror: mirror source must be a contiguous block of p");
    if ((j.transpose & 2) && (((j.transpose & 1) ? j.cols : j.rows) % 128))   // x3_limb_off: N % 128
      return lgx_fail(LGX_EINVAL, "lgx_adam_clip_mirror: a limb mirror needs output rows % 128 == 0");
    const uint64_t rc = (uint64_t)j.rows * j.cols;
    if ((uint64_t)count * rc >= (1ULL << 40))
      return lgx_fail(LGX_EINVAL, "lgx_adam_clip_mirror: mirror block too large for the index arithmetic");
    M.mj[q] = Mirror{off, j.dst_ld, j.dst_bs, j.dst, (int32_t)count, j.rows, j.cols, j.transpose,
                     ((1ULL << 40) + rc - 1) / rc, ((1ULL << 40) + (uint64_t)j.cols - 1) / (uint64_t)j.cols};
  }
  if (!presummed)
    hipLaunchKernelGGL(sumsq_kernel, dim3(nparts), dim3(TPB), 0, LGX_STREAM(stream), g, n, grad_scale, partials, step);
  int blocks = (int)std::min<int64_t>((n + TPB - 1) / TPB, 1024);
  hipLaunchKernelGGL(adam_clip_kernel, dim3(blocks), dim3(TPB), 0, LGX_STREAM(stream), p, g, m, v, n, partials, nparts,
                     grad_scale, max_norm, lr, step, beta1, beta2, eps, M);
  return lgx_hip_status("lgx_adam_clip_mirror");
}

extern "C" int lgx_adam_clip_mirror(float* p, float* g, float* m, float* v, int64_t n, float* partials, int32_t nparts,
                                    float grad_scale, float max_norm, const double* lr, int64_t* step, float beta1,
                                    float beta2, float eps, const lgx_copy2d_job* mirrors, int32_t nmirrors,
                                    void* stream) {
  return adam_clip_mirror_launch(p, g, m, v, n, partials, nparts, grad_scale, max_norm, lr, step, beta1, beta2, eps,
                                 mirrors, nmirrors, stream, false);
}

extern "C" int lgx_adam_clip_mirror_sq(float* p, float* g, float* m, float* v, int64_t n, const float* sq,
                                       int32_t nsq, float max_norm, const double* lr, int64_t* step, float beta1,
                                       float beta2, float eps, const lgx_copy2d_job* mirrors, int32_t nmirrors,
                                       void* stream) {
  return adam_clip_mirror_launch(p, g, m, v, n, const_cast<float*>(sq), nsq, 1.0f, max_norm, lr, step, beta1, beta2,
                                 eps, mirrors, nmirrors, stream, true);
}
