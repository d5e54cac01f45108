// Fused MLP forward on split-bf16 MFMA for the rollout's actor and critic (rsl_rl
// ActorCritic.act / evaluate, obs-512-256-128-{12,1} with ELU: the per-env-step policy
// inference of OnPolicyRunner.learn's rollout loop), both networks in ONE launch (blockIdx.y).
// Same arithmetic as the PPO-update GEMMs (lgx_gemm_split.hip): every f32 operand as three RNE
// bf16 limbs, the six limb products of order <= 2 on v_mfma_f32_32x32x16_bf16 with f32
// accumulation (f32-accurate); 2.67x the product rate of lgx_mlp_forward_kernel's f32 MFMA.
//
//   * 32 rows per workgroup, 8 waves.  The rows' activations stay in LDS across all layers as
//     bf16 limb images [limb][32 rows][Kp] (Kp = width rounded up to 64, 16-byte row pad), split
//     once by their producer (the input staging or the previous layer's epilogue), so the MFMA
//     operand reads are plain ds_read_b128 with no per-fragment split;
//   * weights pre-split (lgx_mlp_x3_split, once per parameter version) into the fragment image
//     [n / 32][k / 16][limb][32 n][16 k]: each wave-load of a fragment limb is 1 KB contiguous,
//     streamed from L2 (a network's limbs are 1.7 MB) with a double-buffered group of k blocks in
//     flight ahead of the MFMAs;
//   * wave w owns output column blocks w, w + 8, ...; the weights are the MFMA's first operand,
//     which leaves each lane four runs of 4 consecutive output columns of one row: bias + ELU +
//     split into 8-byte stores of the next layer's limb image (last layer: f32 rows to HBM).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "lgx_device.h"
#include "lgx_internal.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int XM_BM = 32;           // rows per workgroup
constexpr int XM_NW = 8;            // waves per workgroup
constexpr int XM_NT = 64 * XM_NW;
constexpr int XM_MAXL = 6;
constexpr int XM_MAXW = 512;
constexpr int XM_LDS_MAX = 160 * 1024;
constexpr int XM_ACT_A = 16;        // act epilogue: action columns per row in LDS (LGX_PPO_MAX_ACTIONS)
constexpr int XM_ACT_LDS = (2 * XM_BM * XM_ACT_A + XM_ACT_A) * 4;   // means, draws (then log-prob terms), std

__host__ __device__ inline int xm_kp(int k) { return (k + 63) & ~63; }         // padded width (image / weight K)
__host__ __device__ inline int xm_rs(int k) { return xm_kp(k) * 2 + 16; }       // image row stride, bytes
__host__ __device__ inline int xm_img(int k) { return 3 * XM_BM * xm_rs(k); }   // limb image bytes
__host__ __device__ inline int xm_bp(int n) { return (n + 31) & ~31; }         // bias floats of a layer in LDS

struct XmNet {
  const float* x;
  float* y;
  int64_t rows;
  int32_t nl, act;
  int32_t dims[XM_MAXL + 1];
  const uint16_t* w[XM_MAXL];
  const float* b[XM_MAXL];
};
struct XmBatch {
  XmNet m[2];
  int32_t region;   // byte offset of the second image region (the first at 0)
  int32_t bias_region;   // byte offset of the biases (each layer's zero-padded to 32 columns)
  int32_t act_region;    // byte offset of the act epilogue's rows (lgx_mlp_x3_forward_act)
};
// rsl_rl PPO.act + RolloutStorage.add_transitions (+ the previous step's process_env_step) fused
// into the rollout launch (lgx_mlp_x3_forward_act): the actor's wave 0 finishes its rows in the last
// layer's epilogue (lgx_ppo_act's arithmetic, the same helpers); the waves a late layer leaves idle
// copy the observation rows into storage (actor) and the critic rows + the store (critic)
struct XmAct {
  lgx_ppo_act_args a;
  lgx_ppo_store_args s;
  int32_t store;
};

__device__ __forceinline__ void split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  lgx_split2(x0, x1, l0, l1, l2);   // (lgx_internal.h)
}

template <int ACT>
__device__ __forceinline__ float xm_act_c(float v) {
  if constexpr (ACT == 1) return lgx_elu(v);
  else if constexpr (ACT == 2) return tanhf(v);
  else return v;
}

// One load group of a wave's weight fragments: G = 4 / TPW k blocks x TPW column blocks x 3 limbs
// (12 registers of 16 bytes for TPW 1 or 2), k blocks kb0 .. kb0 + G - 1
constexpr int XM_PF = 12;

template <int TPW>
__device__ __forceinline__ void xm_load(bf16x8 (&b)[XM_PF], const char* __restrict__ W, int KB, int kb0, int wave,
                                        int lane) {
  constexpr int G = 4 / TPW;
  const int lo = (lane & 31) * 32 + (lane >> 5) * 16;     // B fragment lane offset in a 1 KB limb block
#ifdef XM_NO_WLOAD   // A/B: no weight stream (wrong results; measures the MFMA + LDS side alone)
#pragma unroll
  for (int i = 0; i < XM_PF; ++i) b[i] = __builtin_bit_cast(bf16x8, make_uint4(lo + kb0, i, wave, KB));
  return;
#endif
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int l = 0; l < 3; ++l)
        b[(g * TPW + t) * 3 + l] = *reinterpret_cast<const bf16x8*>(
            W + ((int64_t)((wave + XM_NW * t) * KB + kb0 + g) * 3 + l) * 1024 + lo);
}

// column blocks of this wave in a layer of N outputs (wave w owns blocks w, w + 8; N <= 512)
__device__ __forceinline__ int xm_tpw(int N, int wave) {
  const int ncb = (N + 31) / 32;
  return wave < ncb ? (ncb - wave + XM_NW - 1) / XM_NW : 0;
}

// Layer l's first load group, issued ahead of the work before its products (the input staging for
// layer 0, the previous layer's epilogue and barrier otherwise): the weights do not depend on the
// activations, so the L2 latency of each layer's first fragments hides under that work.
__device__ __forceinline__ void xm_prefetch(bf16x8 (&b)[XM_PF], const XmNet& a, int l, int wave, int lane) {
  const int tpw = xm_tpw(a.dims[l + 1], wave), KB = xm_kp(a.dims[l]) / 16;
  const char* W = reinterpret_cast<const char*>(a.w[l]);
  if (tpw == 2) xm_load<2>(b, W, KB, 0, wave, lane);
  else if (tpw == 1) xm_load<1>(b, W, KB, 0, wave, lane);
}

// One layer's products for the TPW column blocks of this wave: acc[t] (+)= W[cb_t] . X over KB
// k blocks of 16 (KB % 4 == 0).  G k blocks per load group, two groups of B fragments in flight;
// bA arrives holding group 0 (xm_prefetch).
template <int TPW>
__device__ __forceinline__ void xm_layer(const char* __restrict__ img, int rs, const char* __restrict__ W, int KB,
                                         int wave, int lane, f32x16 (&acc)[2], bf16x8 (&bA)[XM_PF]) {
  constexpr int G = 4 / TPW;
  const int ao = (lane & 31) * rs + (lane >> 5) * 16;     // A fragment lane offset in an image limb
  const int limb_bytes = XM_BM * rs;
  bf16x8 bB[XM_PF];
  auto compute = [&](const bf16x8 (&b)[XM_PF], int kb0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const char* pa = img + ao + (kb0 + g) * 32;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(pa);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(pa + limb_bytes);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(pa + 2 * limb_bytes);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const bf16x8* w = b + (g * TPW + t) * 3;
        f32x16 c = acc[t];   // small limb products first
#ifdef XM_NO_MFMA   // A/B: weight stream + A reads only (wrong results)
        c[0] += (float)w[2][0] + (float)w[1][1] + (float)w[0][2] + (float)a0[0] + (float)a1[1] + (float)a2[2];
        acc[t] = c;
        continue;
#endif
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], a2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], a0, c, 0, 0, 0);
        acc[t] = c;
      }
    }
  };
  for (int kb0 = 0; kb0 < KB; kb0 += 2 * G) {
    if (kb0 + G < KB) xm_load<TPW>(bB, W, KB, kb0 + G, wave, lane);
    compute(bA, kb0);
    if (kb0 + G >= KB) break;
    if (kb0 + 2 * G < KB) xm_load<TPW>(bA, W, KB, kb0 + 2 * G, wave, lane);
    compute(bB, kb0 + G);
  }
}

template <bool ACT>
__global__ void __launch_bounds__(XM_NT) lgx_mlp_x3_kernel(XmBatch batch, int32_t count, XmAct xa) {
  extern __shared__ __attribute__((aligned(16))) char xm_lds[];
  // two networks: XCDs 0-3 (workgroup id % 8) run the first, 4-7 the second, so each XCD's L2
  // holds one network's weight limbs (1.7 MB) instead of both
  const int b = blockIdx.x;
  const int net = count == 2 ? (b & 7) >> 2 : 0;
  const int64_t tile = count == 2 ? (int64_t)(b >> 3) * 4 + (b & 3) : b;
  const XmNet& a = batch.m[net];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t r0 = tile * XM_BM;
  if (r0 >= a.rows) return;   // (the other network of the launch may have more rows)
  char* const img0 = xm_lds;
  char* const img1 = xm_lds + batch.region;
  float* const bias_lds = reinterpret_cast<float*>(xm_lds + batch.bias_region);
  float* const act_lds = reinterpret_cast<float*>(xm_lds + batch.act_region);   // [32][16] means
  float* const eps_lds = act_lds + XM_BM * XM_ACT_A;                             // [32][16] draws
  float* const sd_lds = eps_lds + XM_BM * XM_ACT_A;                              // [16] std
  if constexpr (ACT) {   // the act epilogue's draws and std, staged with the input rows (clamped loads)
    static_assert(XM_BM * XM_ACT_A <= XM_NT, "one draw per thread");
    if (net == 0) {
      const int A = (int)xa.a.num_actions, rr = tid / XM_ACT_A, c = tid % XM_ACT_A;
      const int64_t gr = std::min<int64_t>(r0 + rr, a.rows - 1);
      const float e = xa.a.noise[gr * A + std::min(c, A - 1)];
      const float sd = xa.a.std[std::min(c, A - 1)];
      eps_lds[tid] = e;
      if (tid < XM_ACT_A) sd_lds[tid] = sd;
    }
  }
  LGX_CLK_DECL(8)
  bf16x8 pre[XM_PF];   // the next layer's first weight load group (xm_prefetch)
  xm_prefetch(pre, a, 0, wave, lane);
  // biases -> LDS (read by the epilogues, not held in registers across the products): this
  // thread's XM_BU entries of the concatenated zero-padded bias rows, loaded with the input rows
  float bvals[XM_MAXL];   // entry tid of each layer's bias row (XM_MAXW <= XM_NT)
  static_assert(XM_MAXW <= XM_NT, "one bias entry per thread and layer");
#pragma unroll
  for (int l = 0; l < XM_MAXL; ++l) {   // clamped, unconditional loads (a per-lane load condition
    if (l < a.nl) {                         // costs a vmcnt(0) round trip per load; §4 of DESIGN.md)
      const float b = a.b[l][min(tid, a.dims[l + 1] - 1)];
      bvals[l] = tid < a.dims[l + 1] ? b : 0.f;
    }
  }
  // ---- input rows -> limb image 0 (zero rows past M, zero columns past K0); XM_SU pairs per
  // thread loaded before any is split, so their HBM latencies overlap
  {
    constexpr int XM_SU = 8;
    const int K0 = a.dims[0], rs = xm_rs(K0), pairs = xm_kp(K0) / 2, total = XM_BM * pairs;
    float* const st_rows = !ACT ? nullptr : net == 0 ? xa.a.st_obs : xa.a.st_cobs;   // (the inputs, host-checked)
    for (int base = 0; base < total; base += XM_SU * XM_NT) {
      float v[XM_SU][2];
#pragma unroll
      for (int u = 0; u < XM_SU; ++u) {
        const int i = base + u * XM_NT + tid;
        const int row = i / pairs, k = 2 * (i - row * pairs);
        const int64_t gr = r0 + row;
        const bool in = i < total && gr < a.rows;
        // clamped, always-valid addresses loaded unconditionally, padding zeroed afterwards
        const int64_t gc = std::min<int64_t>(gr, a.rows - 1) * K0;
        const float x0 = a.x[gc + std::min(k, K0 - 1)], x1 = a.x[gc + std::min(k + 1, K0 - 1)];
        v[u][0] = in && k < K0 ? x0 : 0.f;
        v[u][1] = in && k + 1 < K0 ? x1 : 0.f;
        if constexpr (ACT) {   // RolloutStorage.add_transitions: the observation rows (actor) / the
          if (st_rows && in) {  // critic's rows (privileged observations) into storage row t
            if (k < K0) st_rows[gr * K0 + k] = x0;
            if (k + 1 < K0) st_rows[gr * K0 + k + 1] = x1;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < XM_SU; ++u) {
        const int i = base + u * XM_NT + tid;
        if (i < total) {
          const int row = i / pairs, k = 2 * (i - row * pairs);
          uint32_t l0, l1, l2;
          split2(v[u][0], v[u][1], l0, l1, l2);
          char* p = img0 + row * rs + 2 * k;
          *reinterpret_cast<uint32_t*>(p) = l0;
          *reinterpret_cast<uint32_t*>(p + XM_BM * rs) = l1;
          *reinterpret_cast<uint32_t*>(p + 2 * XM_BM * rs) = l2;
        }
      }
    }
  }
#pragma unroll
  for (int l = 0, off = 0; l < XM_MAXL; ++l) {
    if (l < a.nl) {
      if (tid < xm_bp(a.dims[l + 1])) bias_lds[off + tid] = bvals[l];
      off += xm_bp(a.dims[l + 1]);
    }
  }
  __syncthreads();
  LGX_CLK(0);
  int boff = 0;   // layer l's bias offset in bias_lds
  const int row = lane & 31, h = lane >> 5;
  for (int l = 0; l < a.nl; ++l) {
    const int K = a.dims[l], N = a.dims[l + 1];
    const bool last = l == a.nl - 1;
    const char* in = (l & 1) ? img1 : img0;
    char* out = (l & 1) ? img0 : img1;
    const int ncb = (N + 31) / 32;
    const int tpw = xm_tpw(N, wave);   // column blocks of this wave
    f32x16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
    const char* W = reinterpret_cast<const char*>(a.w[l]);
    if (tpw == 2) xm_layer<2>(in, xm_rs(K), W, xm_kp(K) / 16, wave, lane, acc, pre);
    else if (tpw == 1) xm_layer<1>(in, xm_rs(K), W, xm_kp(K) / 16, wave, lane, acc, pre);
    if (!last) xm_prefetch(pre, a, l + 1, wave, lane);
    LGX_CLK(1 + (l < 4 ? l : 3));
    // epilogue: lane holds row `row`, columns cb*32 + 8q + 4h + (0..3) in acc[t][4q .. 4q+3]
    const int rs_out = xm_rs(N);
    // (the activation is dispatched once per layer, not per value: a per-value test of a.act
    // reloaded it from the kernel arguments with an lgkmcnt(0) wait behind the LDS stores)
    auto epilogue = [&](auto act_c) {
      constexpr int AC = decltype(act_c)::value;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t >= tpw) break;
        const int cb = wave + XM_NW * t;
        // the block's four bias quads read before any image store: the stores may alias the bias
        // rows as far as the compiler knows, so a read after them waits for all of them
        float4 bqs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bqs[q] = *reinterpret_cast<const float4*>(bias_lds + boff + cb * 32 + 8 * q + 4 * h);   // (zero past N)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c0 = cb * 32 + 8 * q + 4 * h;
          float v[4];
          const float4 bq = bqs[q];
          v[0] = acc[t][4 * q] + bq.x;
          v[1] = acc[t][4 * q + 1] + bq.y;
          v[2] = acc[t][4 * q + 2] + bq.z;
          v[3] = acc[t][4 * q + 3] + bq.w;
          if (!last) {   // padding columns: zero weights and bias -> act(0) = 0
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = xm_act_c<AC>(v[i]);
            uint32_t a0, a1, a2, b0, b1, b2;
            split2(v[0], v[1], a0, a1, a2);
            split2(v[2], v[3], b0, b1, b2);
            char* p = out + row * rs_out + 2 * c0;
            *reinterpret_cast<uint2*>(p) = make_uint2(a0, b0);
            *reinterpret_cast<uint2*>(p + XM_BM * rs_out) = make_uint2(a1, b1);
            *reinterpret_cast<uint2*>(p + 2 * XM_BM * rs_out) = make_uint2(a2, b2);
          } else {
            const int64_t gr = r0 + row;
            if (gr < a.rows) {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (c0 + i < N) a.y[gr * N + c0 + i] = v[i];
            }
            if (ACT && net == 0 && c0 < XM_ACT_A)   // the means for the act epilogue
              *reinterpret_cast<float4*>(act_lds + row * XM_ACT_A + c0) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    };
    if (!last && a.act == 1) epilogue(std::integral_constant<int, 1>{});
    else if (!last && a.act == 2) epilogue(std::integral_constant<int, 2>{});
    else epilogue(std::integral_constant<int, 0>{});   // (the output layer has no activation)
    if (!last) {   // image columns past the column blocks (up to the 64-padded width) are zero
      const int c_lo = ncb * 32, kpo = xm_kp(N);
      const int wpairs = (kpo - c_lo) / 2;
      for (int i = tid; i < 3 * XM_BM * wpairs; i += XM_NT) {
        const int lr = i / wpairs, k = c_lo + 2 * (i - lr * wpairs);   // lr = limb * 32 + row
        *reinterpret_cast<uint32_t*>(out + lr * rs_out + 2 * k) = 0u;
      }
    }
    boff += xm_bp(N);
    LGX_CLK(5);
    __syncthreads();   // the output image is complete; the input region is free for the next layer
    LGX_CLK(6);
  }
  if constexpr (ACT) {
    const XmAct* xp = &xa;
    if (net == 1 && xp->store && tid < XM_BM && r0 + tid < a.rows) {   // the previous step's process_env_step rows
      const lgx_ppo_store_args& ps = xp->s;
      const int64_t n = r0 + tid;
      ps.st_rew[n] = ps.time_outs ? lgx_ppo_reward(ps.rew[n], ps.gamma, ps.st_values[n], ps.time_outs[n] != 0)
                                  : ps.rew[n];
      ps.st_dones[n] = ps.reset[n] ? 1 : 0;
    }
    // lgx_ppo_act's arithmetic on the actor's rows (ppo_act_kernel: one thread per (env, action),
    // then the log-prob summed per env in action order) from the means / draws / std in LDS
    if (net == 0) {
      const lgx_ppo_act_args& p = xp->a;
      const int A = (int)p.num_actions, nr = (int)std::min<int64_t>(XM_BM, a.rows - r0);
      const int rr = tid / XM_ACT_A, c = tid % XM_ACT_A;
      if (rr < nr && c < A) {
        const int64_t e = (r0 + rr) * A + c;
        const float mu = act_lds[tid], sd = sd_lds[c];
        const float act = lgx_ppo_sample(mu, sd, eps_lds[tid]);
        p.actions_out[e] = act;
        p.st_actions[e] = act;
        p.st_mu[e] = mu;
        p.st_sigma[e] = sd;
        eps_lds[tid] = lgx_ppo_logp_term(act - mu, sd);
      }
      __syncthreads();
      if (tid < nr) {
        float logp = 0.f;
        for (int j = 0; j < A; ++j) logp += eps_lds[tid * XM_ACT_A + j];
        p.st_logp[r0 + tid] = logp;
      }
    }
  }
  LGX_CLK_PRINT("mlp_x3", 7)
}

// weights W [n_out][k_in] (nn.Linear layout) -> fragment image [n/32][k/16][limb][32 n][16 k],
// zero-padded to 32 n and 64 k; one thread per (n, k pair)
// every layer of a network in one launch (blockIdx.y = layer): one launch per parameter version
// and network instead of one per layer
struct XmSplitJobs {
  const float* W[XM_MAXL];
  uint16_t* dst[XM_MAXL];
  int32_t N[XM_MAXL], K[XM_MAXL];
};

__device__ __forceinline__ void xm_split_one(const float* __restrict__ W, int N, int K, uint16_t* __restrict__ dst,
                                             int64_t i);

__global__ void __launch_bounds__(256) xm_split_kernel(XmSplitJobs J) {
  const int l = blockIdx.y;
  xm_split_one(J.W[l], J.N[l], J.K[l], J.dst[l], (int64_t)blockIdx.x * 256 + threadIdx.x);
}

__device__ __forceinline__ void xm_split_one(const float* __restrict__ W, int N, int K, uint16_t* __restrict__ dst,
                                             int64_t i) {
  const int KP = xm_kp(K), KB = KP / 16, pairs = KP / 2;
  const int64_t total = (int64_t)((N + 31) / 32) * 32 * pairs;
  if (i >= total) return;
  const int n = (int)(i / pairs), k = 2 * (int)(i - (int64_t)n * pairs);
  const float v0 = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
  const float v1 = (n < N && k + 1 < K) ? W[(int64_t)n * K + k + 1] : 0.f;
  uint32_t l0, l1, l2;
  split2(v0, v1, l0, l1, l2);
  const int64_t base = ((int64_t)((n >> 5) * KB + (k >> 4)) * 3) * 512 + (n & 31) * 16 + (k & 15);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst + base);
  d[0] = l0;
  d[256] = l1;   // + 512 bf16 per limb
  d[512] = l2;
}

int64_t lds_bytes(const lgx_mlp_x3_desc* d, int32_t count, int32_t* region, int32_t* bias_region = nullptr,
                  int32_t* act_region = nullptr, bool act = false) {
  int64_t r0 = 0, r1 = 0, rb = 0;
  for (int i = 0; i < count; ++i) {
    const lgx_mlp_x3_desc& m = d[i];
    if (m.nl < 1 || m.nl > XM_MAXL || m.rows < 0 || m.act < 0 || m.act > 2) return -1;
    for (int l = 0; l <= m.nl; ++l)
      if (m.dims[l] <= 0 || m.dims[l] > XM_MAXW) return -1;
    int64_t bb = 0;
    for (int l = 0; l < m.nl; ++l) bb += 4 * xm_bp(m.dims[l + 1]);
    rb = std::max(rb, bb);
    for (int l = 0; l < m.nl; ++l) {   // the image of width dims[l] lives in region l & 1
      const int64_t b = xm_img(m.dims[l]);
      if (l & 1) r1 = std::max(r1, b);
      else r0 = std::max(r0, b);
    }
  }
  if (region) *region = (int32_t)r0;
  if (bias_region) *bias_region = (int32_t)(r0 + r1);
  if (act_region) *act_region = (int32_t)(r0 + r1 + rb);
  const int64_t total = r0 + r1 + rb + (act ? XM_ACT_LDS : 0);
  return total <= XM_LDS_MAX ? total : -1;
}

}  // namespace

extern "C" int64_t lgx_mlp_x3_weight_elems(int32_t n_out, int32_t k_in) {
  if (n_out <= 0 || k_in <= 0) return -1;
  return (int64_t)((n_out + 31) / 32) * (xm_kp(k_in) / 16) * 3 * 512;
}

extern "C" int lgx_mlp_x3_split_layers(const float* const* W, const int32_t* dims, int32_t nl, uint16_t* const* dst,
                                       void* stream) {
  if (!W || !dims || !dst || nl < 1 || nl > XM_MAXL) return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_split: bad layer count");
  XmSplitJobs J{};
  int64_t most = 0;
  for (int l = 0; l < nl; ++l) {
    const int32_t k_in = dims[l], n_out = dims[l + 1];
    if (!W[l] || !dst[l] || n_out <= 0 || k_in <= 0 || n_out > XM_MAXW || k_in > XM_MAXW || ((uintptr_t)dst[l] & 3))
      return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_split: bad args");
    J.W[l] = W[l];
    J.dst[l] = dst[l];
    J.N[l] = n_out;
    J.K[l] = k_in;
    most = std::max<int64_t>(most, (int64_t)((n_out + 31) / 32) * 32 * (xm_kp(k_in) / 2));
  }
  hipLaunchKernelGGL(xm_split_kernel, dim3((unsigned)((most + 255) / 256), (unsigned)nl), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), J);
  return lgx_hip_status("lgx_mlp_x3_split");
}

extern "C" int lgx_mlp_x3_split(const float* W, int32_t n_out, int32_t k_in, uint16_t* dst, void* stream) {
  const int32_t dims[2] = {k_in, n_out};
  return lgx_mlp_x3_split_layers(&W, dims, 1, &dst, stream);
}

extern "C" int64_t lgx_mlp_x3_lds_bytes(const lgx_mlp_x3_desc* d, int32_t count) {
  if (!d || count < 1 || count > 2) return -1;
  return lds_bytes(d, count, nullptr);
}

namespace {
int mlp_x3_launch(const lgx_mlp_x3_desc* d, int32_t count, const XmAct* xa, void* stream) {
  if (!d || count < 1 || count > 2) return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward: count must be 1 or 2");
  XmBatch b{};
  const int64_t lds = lds_bytes(d, count, &b.region, &b.bias_region, &b.act_region, xa != nullptr);
  if (lds < 0) return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward: bad dims or activations exceed the LDS (160 KB)");
  int64_t rows = 0;
  for (int i = 0; i < count; ++i) {
    const lgx_mlp_x3_desc& m = d[i];
    if (!m.x || !m.y) return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward: null rows");
    for (int l = 0; l < m.nl; ++l)
      if (!m.weights[l] || !m.biases[l] || ((uintptr_t)m.weights[l] & 15))
        return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward: weight images must be 16-byte aligned (lgx_mlp_x3_split)");
    XmNet& n = b.m[i];
    n.x = m.x;
    n.y = m.y;
    n.rows = m.rows;
    n.nl = m.nl;
    n.act = m.act;
    for (int l = 0; l <= m.nl; ++l) n.dims[l] = m.dims[l];
    for (int l = 0; l < m.nl; ++l) {
      n.w[l] = m.weights[l];
      n.b[l] = m.biases[l];
    }
    rows = std::max(rows, m.rows);
  }
  if (rows == 0) return LGX_OK;
  static const bool attr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&lgx_mlp_x3_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, XM_LDS_MAX) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&lgx_mlp_x3_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, XM_LDS_MAX) == hipSuccess;
  if (!attr) return lgx_fail(LGX_EHIP, "lgx_mlp_x3_forward: hipFuncSetAttribute (dynamic LDS) failed");
  const int64_t tiles = (rows + XM_BM - 1) / XM_BM;
  const int64_t grid = count == 2 ? 8 * ((tiles + 3) / 4) : tiles;
  if (grid >= (1ll << 31)) return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward: too many rows");
  if (xa) {
    LGX_LAUNCH(lgx_mlp_x3_kernel<true>, dim3((unsigned)grid), dim3(XM_NT), (size_t)lds,
               reinterpret_cast<hipStream_t>(stream), b, count, *xa);
  } else {
    LGX_LAUNCH(lgx_mlp_x3_kernel<false>, dim3((unsigned)grid), dim3(XM_NT), (size_t)lds,
               reinterpret_cast<hipStream_t>(stream), b, count, XmAct{});
  }
  return lgx_hip_status(xa ? "lgx_mlp_x3_forward_act" : "lgx_mlp_x3_forward");
}
}  // namespace

extern "C" int lgx_mlp_x3_forward(const lgx_mlp_x3_desc* d, int32_t count, void* stream) {
  return mlp_x3_launch(d, count, nullptr, stream);
}

extern "C" int lgx_mlp_x3_forward_act(const lgx_mlp_x3_desc* d, int32_t count, const lgx_ppo_act_args* act,
                                      const lgx_ppo_store_args* prev, void* stream) {
  if (!d || count != 2 || !act)
    return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward_act: needs the actor and critic descriptors and act args");
  const lgx_ppo_act_args& p = *act;
  const lgx_mlp_x3_desc &ad = d[0], &cd = d[1];
  if (ad.nl < 1 || ad.nl > XM_MAXL || cd.nl < 1 || cd.nl > XM_MAXL)
    return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward_act: bad layer count");
  if (p.num_envs <= 0 || p.num_envs != ad.rows || p.num_envs != cd.rows || p.num_actions < 1 ||
      p.num_actions > LGX_PPO_MAX_ACTIONS || ad.dims[ad.nl] != p.num_actions || cd.dims[cd.nl] != 1 ||
      p.num_obs <= 0 || !p.std || !p.noise || !p.obs || !p.actions_out || !p.st_obs || !p.st_actions || p.value ||
      !p.st_logp || !p.st_mu || !p.st_sigma || ((p.cobs != nullptr) != (p.st_cobs != nullptr)) ||
      (p.cobs && p.num_cobs <= 0))
    return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward_act: bad act args (rows = envs, actor output = actions <= 16, "
                                "critic output 1, value NULL: the critic writes its storage row)");
  if (p.obs != ad.x || (p.cobs && p.cobs != cd.x) || p.num_obs != ad.dims[0] || (p.cobs && p.num_cobs != cd.dims[0]))
    return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward_act: args->obs / cobs must be the actor / critic inputs");
  XmAct xa{};
  xa.a = p;
  if (prev) {
    const lgx_ppo_store_args& s = *prev;
    if (s.num_envs != p.num_envs || !s.rew || !s.reset || !s.st_values || !s.st_rew || !s.st_dones)
      return lgx_fail(LGX_EINVAL, "lgx_mlp_x3_forward_act: bad store args (the store must cover the same envs)");
    xa.s = s;
    xa.store = 1;
  }
  return mlp_x3_launch(d, count, &xa, stream);
}
