// Internal (non-ABI) declarations shared by the lgx HIP translation units.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "../../include/lgx.h"

#define LGX_MAX_LANE_PTS 24   // contact candidates per leg lane (Go1: 23)

// device-resident model: the ABI model + the per-lane (per-leg) contact candidate tables
struct lgx_dev_model {
  lgx_model m;
  int32_t lane_npts[4];
  int32_t max_lane_npts;
  int32_t joint_rot_eye;   // every joint frame rotation is the identity (URDF rpy = 0: the quadrupeds but ANYmal C)
  int32_t lane_pts[4][LGX_MAX_LANE_PTS];
  int32_t pad_tail[(4 - (sizeof(lgx_model) / 4 + 6 + 4 * LGX_MAX_LANE_PTS) % 4) % 4];   // 16-byte multiple
};

int lgx_launch_ground_contact(const lgx_env_params* dp, const lgx_buffers& b, const float* q, int32_t n, float* o,
                              hipStream_t stream);
int lgx_physics_pp(int32_t n_envs);   // lanes per leg of the physics launch at n_envs (LGX_PHYS_PP overrides)
// frozen != 0: only the drive inputs of `nsub` substeps (clip, targets, actuator-net history and
// model_ins rows) with the state held fixed (lgx_drive_inputs)
// pp: lanes per leg (lgx_physics_pp at lgx_sim_create)
int lgx_launch_physics(const lgx_dev_model* dm, const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs,
                       int32_t nsub, int32_t from_actions, const float* act_src, hipStream_t stream, int32_t frozen,
                       int pp);
// the dense joint-space kernel (lgx_physics.hip): leg_dof == 6 robots, or any with LGX_PHYS_DENSE=1
int lgx_launch_physics_dense(const lgx_dev_model* dm, const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs,
                             int32_t nsub, int32_t from_actions, const float* act_src, hipStream_t stream,
                             int32_t frozen, int32_t num_points);
int lgx_launch_post_physics(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int32_t num_obs,
                            int32_t n_term_rows, int32_t measure_heights, int64_t step, const float* draws,
                            float* extras_snapshot, hipStream_t stream);
// post-physics + the Go1 actuator net (act_rows rows of act_in -> act_out) in one launch
int lgx_launch_post_physics_act(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int64_t step,
                                const float* draws, float* extras_snapshot, const float* act_in, float* act_out,
                                int64_t act_rows, const float* act_w, const float* act_scale, hipStream_t stream);
int lgx_launch_reset_idx(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int32_t n_term_rows,
                         const int32_t* ids, int32_t n, int64_t step, int32_t init_done, const float* draws,
                         float* extras_snapshot, hipStream_t stream);
// wg_per_cu: persistent workgroups per CU of the weight-stationary kernel (2 when it owns the
// chip, 1 when it shares the CUs with concurrent work on another stream)
int lgx_launch_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale,
                            hipStream_t stream, int wg_per_cu = 2);
int lgx_launch_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w,
                             hipStream_t stream);
int lgx_launch_mlp_forward(const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims,
                           const float* const* weights, const float* const* biases, int32_t act, hipStream_t stream);

int lgx_launch_mlp_forward2(const lgx_mlp_desc* d, int32_t count, hipStream_t stream);
int lgx_launch_gae(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                   float* adv, int32_t T, int32_t N, float gamma, float lam, hipStream_t stream);
int lgx_launch_gae_parts(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                         float* adv, int32_t T, int32_t N, float gamma, float lam, double* parts, hipStream_t stream);
int lgx_launch_adv_norm(float* adv, int64_t n, const double* parts, int32_t nparts, hipStream_t stream);
int lgx_launch_gae_norm(const float* rew, const float* val, const uint8_t* dones, const float* last_val, float* ret,
                        float* adv, int32_t T, int32_t N, float gamma, float lam, double* scratch, hipStream_t stream);

// Kernel-tight timing for lgx_profile_*: when the caller arms a (start, stop) event pair, the
// next LGX_LAUNCH on this thread is dispatched with hipExtLaunchKernelGGL, which records the
// events on the kernel's own dispatch (no host launch latency inside the interval).
struct lgx_timing_slot { hipEvent_t start = nullptr, stop = nullptr; };
extern thread_local lgx_timing_slot lgx_timing;
#define LGX_LAUNCH(kern, grid, block, shmem, stream, ...)                                          \
  do {                                                                                           \
    if (lgx_timing.start || lgx_timing.stop) {                                                   \
      hipExtLaunchKernelGGL(kern, grid, block, shmem, stream, lgx_timing.start, lgx_timing.stop, 0, \
                            __VA_ARGS__);                                                        \
      lgx_timing = lgx_timing_slot{};                                                            \
    } else {                                                                                     \
      hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                         \
    }                                                                                            \
  } while (0)

// Pre-split (split-bf16) GEMM operand layout: the LDS image of every 128-column x 32-k block,
// [n / 128][k / 32][limb][n % 128][32 k], the four 16-byte k-chunks of a 64-byte row stored at
// chunk ^ ((n >> 2) & 3) so the 32x32x16 fragment reads (ds_read_b128) are bank-conflict free.
// Offset (bf16 units) of element (n, k) limb `limb` within one batch entry; kb = ceil(K / 32).
// One batch entry holds N * kb * 96 elements (lgx_split_bf16_elems); N % 128 == 0.
__host__ __device__ inline int64_t x3_limb_off(int n, int k, int limb, int kb) {
  const int nn = n & 127, kk = k & 31;
  return ((int64_t)((n >> 7) * kb + (k >> 5)) * 3 + limb) * (128 * 32) + nn * 32 +
         ((((kk >> 3) ^ ((nn >> 2) & 3))) << 3) + (kk & 7);
}

// error reporting shared by the translation units (thread-local message, lgx_last_error)
int lgx_fail(int code, const char* msg);
// lgx_gemm_split.hip: the split-bf16 path of lgx_gemm_nt (arguments already checked)
int lgx_gemm_nt_split(const lgx_gemm_args& a, int cus, void* stream);
// lgx_gemm_x3p.hip: pipelined split-bf16 path (pre-split B, K % 32 == 0)
int lgx_gemm_nt_x3p(const lgx_gemm_args& a, int cus, void* stream);
int lgx_hip_status(const char* what);  // LGX_OK or LGX_EHIP from hipGetLastError()

// a batch of reduction jobs passed by value to one launch (lgx_reduce_slices)
struct lgx_reduce_jobs {
  lgx_reduce_job job[LGX_MAX_REDUCE_JOBS];
  int32_t tile_start[LGX_MAX_REDUCE_JOBS];    // first tile of each job in the flat grid
  int32_t tile_outputs[LGX_MAX_REDUCE_JOBS];  // outputs per tile (16 or 64)
};

// scratch layout (floats): [blocks][LGX_MAX_TERMS + 2] reduction partials
#ifndef LGX_ENV_BLOCK
#define LGX_ENV_BLOCK 16  // envs per post-physics workgroup (16 lanes each)
#endif
#define LGX_PARTIAL_STRIDE (LGX_MAX_TERMS + 2)

#ifdef __HIPCC__
// ELU (alpha 1) of the policy networks: exp(x) - 1 on v_exp_f32 for x <= 0.  Absolute error
// <= ~1.2e-7 against torch's expm1 (a few ulp of 1; relative error grows only where the output
// is tiny, |x| < 2^-8); libm's expm1f costs ~10x more VALU, which in the GEMM epilogues competes
// with the operand splits for the MFMA issue gaps (measured: layer-1 forward 54 -> 61 us with
// an expm1-accurate polynomial form).
__device__ __forceinline__ float lgx_elu(float x) { return x > 0.f ? x : __expf(x) - 1.f; }
// Normal(mu, sd).sample() from a standard-normal draw (torch.normal = normal_(0, 1) * std + mu) and
// the log-prob term of one action dimension (Normal.log_prob); shared by lgx_ppo_act and the
// rollout MLP's fused act epilogue so both write bit-identical rows.  Explicit fma, no contraction.
__device__ __forceinline__ float lgx_ppo_sample(float mu, float sd, float eps) { return __builtin_fmaf(sd, eps, mu); }
__device__ __forceinline__ float lgx_ppo_logp_term(float d, float sd) {
#pragma clang fp contract(off)
  const float half_log_2pi = 0.91893853320467274178f;
  return -(d * d) / (2.f * sd * sd) - logf(sd) - half_log_2pi;
}
// Three RNE bf16 limbs of two f32 values, packed (low half = first value): x = l0 + l1 + l2 + e,
// |e| <= 2^-24 |x|; both subtractions are exact.  The split-bf16 GEMMs' operand split (lgx_gemm_x3p
// / _tn / _split, lgx_mlp_x3).  (Round 6 measured the residuals as v_dot2c_f32_bf16 with a -1 in the
// limb's half - 7 VALU per pair instead of 11, bitwise the same limbs - and the PPO update was
// slower, 10.83 vs 10.46 ms, same box, alternated: the dot instruction does not issue at the rate of
// the shift / subtract it replaces.)
typedef __bf16 lgx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float lgx_fx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void lgx_split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  l0 = __builtin_bit_cast(uint32_t, __builtin_convertvector((lgx_fx2){x0, x1}, lgx_bf16x2));
  float r0 = x0 - __uint_as_float(l0 << 16), r1 = x1 - __uint_as_float(l0 & 0xffff0000u);
  l1 = __builtin_bit_cast(uint32_t, __builtin_convertvector((lgx_fx2){r0, r1}, lgx_bf16x2));
  r0 -= __uint_as_float(l1 << 16);
  r1 -= __uint_as_float(l1 & 0xffff0000u);
  l2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((lgx_fx2){r0, r1}, lgx_bf16x2));
}
// PPO.process_env_step's time-out bootstrap: rew + gamma * (V * time_out), as torch evaluates it
__device__ __forceinline__ float lgx_ppo_reward(float rew, float gamma, float value, bool time_out) {
#pragma clang fp contract(off)
  return rew + gamma * (value * (time_out ? 1.f : 0.f));
}
#endif
