// lgx post-physics kernel: the fused LeggedRobot.post_physics_step (legged_robot.py:109-141)
// — base-frame transforms, command resampling / heading, height scan, pushes, termination,
// the reward terms in reference order, reset_idx, observations + noise + clip, last_* copies —
// with no host synchronisation (the reference's reset_buf.nonzero() and per-term launches
// are replaced by per-env predication and a deterministic two-stage reduction for extras).
//
// Block = 16 lanes per env x LGX_ENV_BLOCK envs.  Phases:
//   A  (all lanes) height scan: (env, point) pairs, coalesced int16 gathers
//   B  (one lane per env) scalar env logic: scalar logic, rewards, reset
//   C  (all lanes) observation rows: (env, obs index) pairs, coalesced stores
// Extras (episode means over reset envs) are reduced per block in LDS, then by the workgroup
// that finishes last, in fixed order (bitwise reproducible).
#include <algorithm>

#include "lgx_device.h"
#include "lgx_internal.h"
#include "lgx_actuator_ws.h"

#define ENV_THREADS (16 * LGX_ENV_BLOCK)
static_assert(LGX_DRAW_NOISE % 4 == 0, "observation noise slots must start a Philox block");

namespace {

struct Draws {
  const lgx_env_params* P;
  const float* inj;  // injected [N, stride] or null
  int32_t stride;
  LGX_DEV float operator()(int e, int slot, int64_t step, uint32_t tag) const {
    return inj ? inj[(int64_t)e * stride + slot] : lgx_uniform(P->seed, e, slot, step, tag);
  }
  // slots 4q .. 4q+3 (one Philox block); injected rows may end mid-block
  LGX_DEV void quad(int e, int q, int64_t step, uint32_t tag, float u[4]) const {
    if (inj) {
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = 4 * q + k < stride ? inj[(int64_t)e * stride + 4 * q + k] : 0.f;
    } else {
      lgx_uniform4(P->seed, e, q, step, tag, u);
    }
  }
};

LGX_DEV float wrap_to_pi(float a) {  // utils/math.py:45-48 (torch remainder semantics)
  const float tp = (float)(2.0 * 3.14159265358979323846);
  float r = fmodf(a, tp);
  if (r != 0.0f && r < 0.0f) r += tp;
  if (r > (float)3.14159265358979323846) r -= tp;
  return r;
}

LGX_DEV void resample_cmd(const lgx_env_params* __restrict__ P, const Draws& D, int e, int slot, int64_t step,
                          uint32_t tag, float* c) {  // legged_robot.py:354-368
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float lo = P->cmd_ranges[k][0], hi = P->cmd_ranges[k][1];
    c[k] = (hi - lo) * D(e, slot + k, step, tag) + lo;
  }
  int k3 = P->heading_command ? 3 : 2;
  float lo = P->cmd_ranges[k3][0], hi = P->cmd_ranges[k3][1];
  float v = (hi - lo) * D(e, slot + 2, step, tag) + lo;
  if (k3 == 3) c[3] = v; else c[2] = v;
  float keep = sqrtf(c[0] * c[0] + c[1] * c[1]) > 0.2f ? 1.0f : 0.0f;
  c[0] *= keep; c[1] *= keep;
}

LGX_DEV float norm3p(const float* f) { return sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]); }

struct EnvView {
  f3 blv, bav, pg;
  float cmd[4];
  const float* ds;   // dof_state row (pre-reset)
  const float* tq;
  const float* cf;
  const float* act;
  const float* la;
  const float* ldv;
  float* fat;
  float rootz;
  const float* mh;
  bool reset, time_out;
};

LGX_DEV float reward_term(const lgx_env_params* __restrict__ P, const EnvView& v, int id) {  // :857-966
  float s = 0.f;
  switch (id) {
    case LGX_R_LIN_VEL_Z: return v.blv.z * v.blv.z;
    case LGX_R_ANG_VEL_XY: return v.bav.x * v.bav.x + v.bav.y * v.bav.y;
    case LGX_R_ORIENTATION: return v.pg.x * v.pg.x + v.pg.y * v.pg.y;
    case LGX_R_BASE_HEIGHT: {
      float acc;
      if (P->measure_heights) {
        acc = 0.f;
        for (int i = 0; i < P->num_height_points; ++i) acc += v.rootz - v.mh[i];
        acc /= (float)P->num_height_points;
      } else acc = v.rootz;
      float d = acc - P->base_height_target;
      return d * d;
    }
    case LGX_R_TORQUES: for (int j = 0; j < 12; ++j) s += v.tq[j] * v.tq[j]; return s;
    case LGX_R_ENERGY: for (int j = 0; j < 12; ++j) { float x = v.tq[j] * v.ds[2 * j + 1]; s += x * x; } return s;
    case LGX_R_DOF_VEL: for (int j = 0; j < 12; ++j) s += v.ds[2 * j + 1] * v.ds[2 * j + 1]; return s;
    case LGX_R_DOF_ACC:
      for (int j = 0; j < 12; ++j) { float x = (v.ldv[j] - v.ds[2 * j + 1]) / P->dt; s += x * x; }
      return s;
    case LGX_R_ACTION_RATE: for (int j = 0; j < 12; ++j) { float x = v.la[j] - v.act[j]; s += x * x; } return s;
    case LGX_R_COLLISION:
      for (int i = 0; i < P->num_penalised; ++i) s += norm3p(v.cf + 3 * P->penalised_indices[i]) > 0.1f ? 1.f : 0.f;
      return s;
    case LGX_R_TERMINATION: return (v.reset && !v.time_out) ? 1.f : 0.f;
    case LGX_R_DOF_POS_LIMITS:
      for (int j = 0; j < 12; ++j) {
        float lo = v.ds[2 * j] - P->soft_lower[j], hi = v.ds[2 * j] - P->soft_upper[j];
        s += -(lo < 0.f ? lo : 0.f) + (hi > 0.f ? hi : 0.f);
      }
      return s;
    case LGX_R_DOF_VEL_LIMITS:
      for (int j = 0; j < 12; ++j)
        s += clampf(fabsf(v.ds[2 * j + 1]) - P->dof_vel_limits[j] * P->soft_dof_vel_limit, 0.f, 1.f);
      return s;
    case LGX_R_TORQUE_LIMITS:
      for (int j = 0; j < 12; ++j) s += fmaxf(fabsf(v.tq[j]) - P->torque_limits[j] * P->soft_torque_limit, 0.f);
      return s;
    case LGX_R_TRACKING_LIN_VEL: {
      float ex = v.cmd[0] - v.blv.x, ey = v.cmd[1] - v.blv.y;
      return expf(-(ex * ex + ey * ey) / P->tracking_sigma);
    }
    case LGX_R_TRACKING_ANG_VEL: { float ez = v.cmd[2] - v.bav.z; return expf(-(ez * ez) / P->tracking_sigma); }
    case LGX_R_FEET_AIR_TIME: {  // mutates feet_air_time (:941-949)
      for (int f = 0; f < P->num_feet; ++f) {
        bool contact = v.cf[3 * P->feet_indices[f] + 2] > 1.0f;
        float first = (v.fat[f] > 0.f && contact) ? 1.f : 0.f;
        v.fat[f] += P->dt;
        s += (v.fat[f] - 0.5f) * first;
      }
      s *= (sqrtf(v.cmd[0] * v.cmd[0] + v.cmd[1] * v.cmd[1]) > 0.1f) ? 1.f : 0.f;
      for (int f = 0; f < P->num_feet; ++f)
        if (v.cf[3 * P->feet_indices[f] + 2] > 1.0f) v.fat[f] = 0.f;
      return s;
    }
    case LGX_R_STUMBLE:
      for (int f = 0; f < P->num_feet; ++f) {
        const float* F = v.cf + 3 * P->feet_indices[f];
        if (sqrtf(F[0] * F[0] + F[1] * F[1]) > 5.f * fabsf(F[2])) return 1.f;
      }
      return 0.f;
    case LGX_R_STAND_STILL:
      for (int j = 0; j < 12; ++j) s += fabsf(v.ds[2 * j] - P->default_dof_pos[j]);
      return s * ((sqrtf(v.cmd[0] * v.cmd[0] + v.cmd[1] * v.cmd[1]) < 0.1f) ? 1.f : 0.f);
    case LGX_R_FEET_CONTACT_FORCES:
      for (int f = 0; f < P->num_feet; ++f) s += fmaxf(norm3p(v.cf + 3 * P->feet_indices[f]) - P->max_contact_force, 0.f);
      return s;
    case LGX_R_HIP_MOTION:
      for (int j = 0; j < 12; j += 3) s += fabsf(v.ds[2 * j] - P->default_dof_pos[j]);
      return s;
    case LGX_R_NO_FLY: {  // Cassie (cassie.py:42-46): exactly one foot with F_z > 0.1 N
      int n = 0;
      for (int f = 0; f < P->num_feet; ++f) n += v.cf[3 * P->feet_indices[f] + 2] > 0.1f ? 1 : 0;
      return n == 1 ? 1.f : 0.f;
    }
  }
  return 0.f;
}

// reset one env (legged_robot.py:150-180, per env); cmd is the env's command row in registers
LGX_DEV void reset_env(const lgx_env_params* __restrict__ P, const lgx_buffers& B, const Draws& D, int e,
                       int64_t step, uint32_t tag, bool init_done, float* cmd) {
  float* org = B.env_origins + (int64_t)e * 3;
  float* rs = B.root_states + (int64_t)e * 13;
  if (P->curriculum && init_done) {  // _update_terrain_curriculum :443-463
    float dx = rs[0] - org[0], dy = rs[1] - org[1];
    float dist = sqrtf(dx * dx + dy * dy);
    bool up = dist > P->terrain_env_length / 2.0f;
    bool down = (dist < sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) * P->max_episode_length_s * 0.5f) && !up;
    int64_t lvl = B.terrain_levels[e] + (up ? 1 : 0) - (down ? 1 : 0);
    if (lvl >= P->max_terrain_level) {
      int64_t r = (int64_t)(D(e, LGX_DRAW_CURRIC, step, tag) * (float)P->max_terrain_level);
      lvl = r >= P->max_terrain_level ? P->max_terrain_level - 1 : r;
    } else if (lvl < 0) lvl = 0;
    B.terrain_levels[e] = lvl;
    const float* to = B.terrain_origins + (lvl * P->terrain_num_cols + B.terrain_types[e]) * 3;
    org[0] = to[0]; org[1] = to[1]; org[2] = to[2];
  }
  float* ds = B.dof_state + (int64_t)e * 24;
  for (int j = 0; j < 12; ++j) {
    ds[2 * j] = P->default_dof_pos[j] * ((1.5f - 0.5f) * D(e, LGX_DRAW_RESET_DOF + j, step, tag) + 0.5f);
    ds[2 * j + 1] = 0.f;
  }
  for (int i = 0; i < 13; ++i) rs[i] = P->base_init_state[i];
  for (int i = 0; i < 3; ++i) rs[i] += org[i];
  if (P->custom_origins)
    for (int i = 0; i < 2; ++i) rs[i] += (1.0f - -1.0f) * D(e, LGX_DRAW_RESET_XY + i, step, tag) + -1.0f;
  for (int i = 0; i < 6; ++i) rs[7 + i] = (0.5f - -0.5f) * D(e, LGX_DRAW_RESET_VEL + i, step, tag) + -0.5f;
  resample_cmd(P, D, e, LGX_DRAW_RESET_CMD, step, tag, cmd);
  for (int j = 0; j < 12; ++j) { B.last_actions[(int64_t)e * 12 + j] = 0.f; B.last_dof_vel[(int64_t)e * 12 + j] = 0.f; }
  for (int f = 0; f < 4; ++f) B.feet_air_time[(int64_t)e * 4 + f] = 0.f;
  if (B.sea_h && B.sea_c) {   // Anymal.reset_idx zeroes the SEA LSTM state (anymal.py:56-60)
    const int64_t m = (int64_t)P->num_envs * 12;
    float4* h = reinterpret_cast<float4*>(B.sea_h);
    float4* c = reinterpret_cast<float4*>(B.sea_c);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int L = 0; L < 2; ++L)
      for (int i = 0; i < 24; ++i) {
        h[((int64_t)L * m + (int64_t)e * 12) * 2 + i] = z;
        c[((int64_t)L * m + (int64_t)e * 12) * 2 + i] = z;
      }
  }
  B.episode_length[e] = 0;
  B.reset[e] = 1;
}

// per-block deterministic partial sums of the episode sums of reset envs (+ reset count)
LGX_DEV void block_partials(float (*lds)[LGX_PARTIAL_STRIDE], int nrows, float* partial_out) {
  __syncthreads();
  int t = threadIdx.x;
  if (t < nrows + 2) {  // term sums, reset count, terrain-level sum
    float s = 0.f;
    for (int i = 0; i < LGX_ENV_BLOCK; ++i) s += lds[i][t];
    partial_out[t] = s;
  }
}

// extras finalize: deterministic sum of the block partials; publish only if >= 1 env reset.
// level_scan: sum terrain levels over all envs here (reset_idx path) instead of partials.
// Runs on one workgroup of nt threads (a multiple of 64).
LGX_DEV void extras_finalize_body(const lgx_env_params* __restrict__ P, const lgx_buffers& B, int32_t nblocks,
                                  int32_t level_scan, float* __restrict__ snapshot, int nt) {
  const int N = P->num_envs;
  const int T = P->num_terms + (P->termination_slot >= 0 ? 1 : 0);
  __shared__ float sums[LGX_PARTIAL_STRIDE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = nt >> 6;
  // wave w reduces rows w, w+nw, ...: lanes take blocks lane, lane+64, ... then a fixed-order
  // butterfly (deterministic, no atomics)
  const int rows = T + 2;
  for (int r = wave; r < rows; r += nw) {
    float s = 0.f;
    if (r == T + 1 && level_scan) {
      if (P->curriculum)
        for (int e = lane; e < N; e += 64) s += (float)B.terrain_levels[e];
    } else {
      for (int b = lane; b < nblocks; b += 64) s += B.scratch[(int64_t)b * LGX_PARTIAL_STRIDE + r];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) sums[r] = s;
  }
  __syncthreads();
  const float count = sums[T];
  const bool update = count > 0.f;  // else the reference keeps stale extras (legged_robot.py:160-161)
  if (t < rows) {
    float v = B.extras[t];
    if (update) {
      if (t < T) v = (sums[t] / count) / P->max_episode_length_s;
      else if (t == T + 1) v = count;
      else if (P->curriculum) v = sums[T + 1] / (float)N;
      B.extras[t] = v;
    }
    if (snapshot) snapshot[t] = v;  // this step's published copy (lgx_rebind_extras)
  }
  if (!update) return;
  if (P->send_timeouts)
    for (int e = t; e < N; e += nt) B.extras_time_outs[e] = B.time_out[e];
}

// Completion ticket of the post-physics workgroups (a counter after the block partials in
// scratch, zero between launches): the workgroup that takes the last ticket runs the extras
// finalize, so the reduction needs no second launch.  Release: every thread's partial /
// time_out / level writes are fenced at device scope before the ticket; acquire: the last
// workgroup fences again before reading them (the L2s of the 8 XCDs are not coherent).
// The release fence (an L2 write-back at agent scope) is taken by wave 0 only: every write the
// finalize reads comes from wave 0 - the block's partial row from threads < T + 2 <= 64
// (block_partials), time_out / extras_time_outs and the curriculum levels from the env lanes
// (threads < LGX_ENV_BLOCK <= 64) - and every other wave skips the write-back (measured: all
// four waves fencing took ~15 us of each workgroup's timeline).
LGX_DEV bool take_last_ticket(const lgx_buffers& B, int nblocks) {
  __shared__ int last;
  static_assert(LGX_PARTIAL_STRIDE <= 64, "the partial-row writers are wave 0");
  static_assert(LGX_ENV_BLOCK <= 64, "the env lanes (time_out, levels) are wave 0");
  if (threadIdx.x < 64) __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int* ctr = reinterpret_cast<unsigned int*>(B.scratch + (int64_t)nblocks * LGX_PARTIAL_STRIDE);
    const unsigned int ticket = atomicAdd(ctr, 1u);
    last = ticket == (unsigned int)nblocks - 1u;
    if (last) atomicExch(ctr, 0u);  // ready for the next launch (stream-ordered after this one)
  }
  __syncthreads();
  if (last) __threadfence();
  return last;
}

// one post-physics workgroup: envs [blk * LGX_ENV_BLOCK, +LGX_ENV_BLOCK) of nblocks
LGX_DEV void post_physics_body(const lgx_env_params* __restrict__ P, const lgx_buffers& B, int64_t step,
                               const float* draws, int blk, int nblocks, float* snapshot) {
  const int N = P->num_envs;
  const int nobs = P->num_obs;
  const int e0 = blk * LGX_ENV_BLOCK;
  const int tid = threadIdx.x;
  const Draws D{P, draws, LGX_DRAW_NOISE + nobs};
  const int T = P->num_terms + (P->termination_slot >= 0 ? 1 : 0);
  LGX_CLK_DECL(6)
  __shared__ float part[LGX_ENV_BLOCK][LGX_PARTIAL_STRIDE];
  // what phase C (observations) reads, kept in LDS: heights (phase A), base-frame velocities,
  // gravity, commands and root z (phase B, post-reset); dof state / actions are in srow below
  __shared__ float sheight[LGX_ENV_BLOCK][LGX_MAX_HEIGHT_POINTS];
  __shared__ float sbase[LGX_ENV_BLOCK][14];   // blv 3, bav 3, pg 3, cmd 4, root z
  // per-observation-index constants (scale, offset, noise scale) and the scan pattern, staged once
  // per workgroup: phases A and C index them per lane, which from global memory is a dependent
  // vector load per entry
  __shared__ float obs_mul[LGX_MAX_OBS], obs_sub[LGX_MAX_OBS], obs_nsc[LGX_MAX_OBS];
  __shared__ float2 scan_pt[LGX_MAX_HEIGHT_POINTS];
  for (int i = tid; i < nobs; i += ENV_THREADS) {
    float mul, sub = 0.f;
    if (i < 3) mul = P->obs_scale_lin_vel;
    else if (i < 6) mul = P->obs_scale_ang_vel;
    else if (i < 9) mul = 1.f;
    else if (i < 12) mul = i < 11 ? P->obs_scale_lin_vel : P->obs_scale_ang_vel;
    else if (i < 24) { mul = P->obs_scale_dof_pos; sub = P->default_dof_pos[i - 12]; }
    else if (i < 36) mul = P->obs_scale_dof_vel;
    else if (i < 48) mul = 1.f;
    else mul = P->obs_scale_height;
    obs_mul[i] = mul;
    obs_sub[i] = sub;
    obs_nsc[i] = P->add_noise ? P->noise_scale_vec[i] : 0.f;
  }
  if (P->measure_heights)
    for (int i = tid; i < P->num_height_points; i += ENV_THREADS)
      scan_pt[i] = make_float2(P->height_points[i][0], P->height_points[i][1]);

  // ---- phase A: height scan (legged_robot.py:818-854), pre-reset base pose.  The per-env yaw
  // rotation and base xy are staged in LDS; the (env, point) loop is unrolled so several
  // heightfield gathers are in flight per lane.
  if (P->measure_heights) {
    __shared__ float4 base_xy_yaw[LGX_ENV_BLOCK];
    if (tid < LGX_ENV_BLOCK) {
      const int e = min(e0 + tid, N - 1);
      const float* rs = B.root_states + (int64_t)e * 13;
      float z = rs[5], w = rs[6];
      float nrm = fmaxf(sqrtf(z * z + w * w), 1e-9f);
      base_xy_yaw[tid] = make_float4(rs[0], rs[1], z / nrm, w / nrm);
    }
    __syncthreads();
    const int np = P->num_height_points;
    const int total = LGX_ENV_BLOCK * np;
    if (P->terrain_kind == 0) {  // plane: zeros (:831-832)
      for (int idx = tid; idx < total; idx += ENV_THREADS) {
        const int le = idx / np, i = idx - le * np;
        if (e0 + le < N) B.measured_heights[(int64_t)(e0 + le) * np + i] = 0.f;
        sheight[le][i] = 0.f;
      }
    } else {
      // every lane gathers (rows past N use the clamped env staged above; only the stores are
      // predicated): a gather inside a branch compiles to one exposed round trip per iteration,
      // unconditional ones let the unrolled iterations' gathers overlap
      const int16_t* H = B.height_samples;
      const int cols = B.hf_cols;
      const float rmax = (float)(B.hf_rows - 2), cmax = (float)(B.hf_cols - 2);
      constexpr int U = 4;  // (env, point) pairs per lane in flight: all gathers issued before any store
      for (int base = tid; base < total; base += U * ENV_THREADS) {
        int hq[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int idx = min(base + u * ENV_THREADS, total - 1);
          const int le = idx / np, i = idx - le * np;
          const float4 b = base_xy_yaw[le];
          const float2 hp = scan_pt[i];
          f3 o = quat_apply(0.f, 0.f, b.z, b.w, mk3(hp.x, hp.y, 0.f));
          float x = o.x + b.x + P->border_size, y = o.y + b.y + P->border_size;  // (p + root) + border, as :833-834
          // .long() truncation then clip to [0, rows - 2] (:835-838) == clamp then truncate
          const int px = (int)fminf(fmaxf(x / P->horizontal_scale, 0.f), rmax);
          const int py = (int)fminf(fmaxf(y / P->horizontal_scale, 0.f), cmax);
          const int16_t* q = H + px * cols + py;
          hq[u][0] = q[0]; hq[u][1] = q[cols]; hq[u][2] = q[1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int idx = base + u * ENV_THREADS;
          if (idx >= total) break;
          const int le = idx / np, i = idx - le * np;
          const float hv = (float)min(min(hq[u][0], hq[u][1]), hq[u][2]) * P->vertical_scale;
          if (e0 + le < N) B.measured_heights[(int64_t)(e0 + le) * np + i] = hv;
          sheight[le][i] = hv;
        }
      }
    }
    __syncthreads();
  }

  LGX_CLK(0);
  // ---- stage the per-env rows the reward terms read (coalesced, all lanes) into LDS: the
  // term loop below re-reads them many times from a single lane per env
  constexpr int SROW = 24 + 12 + LGX_MAX_BODIES * 3 + 12 + 12 + 12;  // ds tq cf act la ldv
  __shared__ float srow[LGX_ENV_BLOCK][SROW + 1];
  {
    // the source address is selected, the load itself is unconditional, and U of them are in
    // flight per lane before the LDS stores (a load per branch arm is one round trip each)
    constexpr int U = 4;
    for (int base = tid; base < LGX_ENV_BLOCK * SROW; base += U * ENV_THREADS) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = min(base + u * ENV_THREADS, LGX_ENV_BLOCK * SROW - 1);
        const int le = idx / SROW, c = idx - le * SROW;
        const int64_t e = min(e0 + le, N - 1);
        const float* src;
        if (c < 24) src = B.dof_state + e * 24 + c;
        else if (c < 36) src = B.torques + e * 12 + c - 24;
        else if (c < 36 + LGX_MAX_BODIES * 3) src = B.contact_forces + e * LGX_MAX_BODIES * 3 + c - 36;
        else if (c < 48 + LGX_MAX_BODIES * 3) src = B.actions + e * 12 + c - 36 - LGX_MAX_BODIES * 3;
        else if (c < 60 + LGX_MAX_BODIES * 3) src = B.last_actions + e * 12 + c - 48 - LGX_MAX_BODIES * 3;
        else src = B.last_dof_vel + e * 12 + c - 60 - LGX_MAX_BODIES * 3;
        v[u] = *src;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * ENV_THREADS;
        if (idx < LGX_ENV_BLOCK * SROW) srow[idx / SROW][idx % SROW] = v[u];
      }
    }
  }
  // the env lane's pre-step root state, commands and episode length, staged with the rows above
  // (their global loads would otherwise be phase B's first exposed round trip)
  __shared__ float sroot[LGX_ENV_BLOCK][13];
  __shared__ float scmd[LGX_ENV_BLOCK][4];
  __shared__ int64_t sep[LGX_ENV_BLOCK];
  for (int idx = tid; idx < LGX_ENV_BLOCK * 17; idx += ENV_THREADS) {
    const int le = idx / 17, c = idx - le * 17;
    const int64_t e = min(e0 + le, N - 1);
    if (c < 13) sroot[le][c] = B.root_states[e * 13 + c];
    else scmd[le][c - 13] = B.commands[e * 4 + c - 13];
  }
  if (tid < LGX_ENV_BLOCK) sep[tid] = B.episode_length[min(e0 + tid, N - 1)];
  // episode sums [T, N] and feet_air_time [N, 4] are read-modify-written by the env lane: stage
  // them too (coalesced over envs), so phase B has no dependent global round trips
  __shared__ float ssum[LGX_MAX_TERMS][LGX_ENV_BLOCK];
  __shared__ float sfat[LGX_ENV_BLOCK][4];
  for (int idx = tid; idx < T * LGX_ENV_BLOCK; idx += ENV_THREADS) {
    const int t = idx / LGX_ENV_BLOCK, le = idx - t * LGX_ENV_BLOCK;
    ssum[t][le] = e0 + le < N ? B.episode_sums[(int64_t)t * N + e0 + le] : 0.f;
  }
  if (tid < LGX_ENV_BLOCK * 4) {
    const int le = tid >> 2;
    sfat[le][tid & 3] = e0 + le < N ? B.feet_air_time[(int64_t)(e0 + le) * 4 + (tid & 3)] : 0.f;
  }
  __syncthreads();

  LGX_CLK(1);
  // ---- phase B: one env per lane
  if (tid < LGX_ENV_BLOCK) {
    const int e = e0 + tid;
    for (int t = 0; t < LGX_PARTIAL_STRIDE; ++t) part[tid][t] = 0.f;
    if (e < N) {
      int64_t ep = sep[tid] + 1;  // :118
      B.episode_length[e] = ep;
      float* rs = B.root_states + (int64_t)e * 13;   // (written: pushes, resets)
      const float* rs0 = sroot[tid];                 // pre-step values, staged
      const float qx = rs0[3], qy = rs0[4], qz = rs0[5], qw = rs0[6];
      EnvView v;
      v.blv = quat_rotate_inverse(qx, qy, qz, qw, mk3(rs0[7], rs0[8], rs0[9]));     // :122-125
      v.bav = quat_rotate_inverse(qx, qy, qz, qw, mk3(rs0[10], rs0[11], rs0[12]));
      v.pg = quat_rotate_inverse(qx, qy, qz, qw, mk3(0.f, 0.f, -1.f));
      float* cmd_g = B.commands + (int64_t)e * 4;
      for (int k = 0; k < 4; ++k) v.cmd[k] = scmd[tid][k];
      if (ep % P->resample_interval == 0) resample_cmd(P, D, e, LGX_DRAW_CMD, step, 0u, v.cmd);  // :342-343
      if (P->heading_command) {  // :344-347
        f3 f = quat_apply(qx, qy, qz, qw, mk3(1.f, 0.f, 0.f));
        float heading = atan2f(f.y, f.x);
        v.cmd[2] = clampf(0.5f * wrap_to_pi(v.cmd[3] - heading), -1.f, 1.f);
      }
      if (P->push_robots && step % P->push_interval == 0) {  // :351-352, 436-441
        float mv = P->max_push_vel_xy;
        rs[7] = (mv - -mv) * D(e, LGX_DRAW_PUSH, step, 0u) + -mv;
        rs[8] = (mv - -mv) * D(e, LGX_DRAW_PUSH + 1, step, 0u) + -mv;
      }
      v.ds = srow[tid];                    // pre-reset rows, staged above
      v.tq = srow[tid] + 24;
      v.cf = srow[tid] + 36;
      v.act = srow[tid] + 36 + LGX_MAX_BODIES * 3;
      v.la = srow[tid] + 48 + LGX_MAX_BODIES * 3;
      v.ldv = srow[tid] + 60 + LGX_MAX_BODIES * 3;
      v.fat = sfat[tid];
      v.rootz = rs0[2];
      v.mh = P->measure_heights ? sheight[tid] : nullptr;   // this step's scan (phase A), from LDS
      // check_termination :143-148
      bool r = false;
      for (int i = 0; i < P->num_termination_bodies; ++i) r |= norm3p(v.cf + 3 * P->termination_indices[i]) > 1.f;
      v.time_out = (float)ep > P->max_episode_length;
      v.reset = r || v.time_out;
      // compute_reward :195-212
      float rew = 0.f;
      for (int t = 0; t < P->num_terms; ++t) {
        float rr = reward_term(P, v, P->term_ids[t]) * P->term_scales[t];
        rew += rr;
        ssum[t][tid] += rr;
      }
      if (P->only_positive_rewards) rew = fmaxf(rew, 0.f);
      if (P->termination_slot >= 0) {
        float rr = reward_term(P, v, LGX_R_TERMINATION) * P->termination_scale;
        rew += rr;
        ssum[P->termination_slot][tid] += rr;
      }
      B.rew[e] = rew;
      B.time_out[e] = v.time_out ? 1 : 0;
      B.reset[e] = v.reset ? 1 : 0;
      if (v.reset) {  // reset_idx :150-193
        for (int t = 0; t < T; ++t) {
          part[tid][t] = ssum[t][tid];
          ssum[t][tid] = 0.f;
        }
        part[tid][T] = 1.f;
        reset_env(P, B, D, e, step, 0u, true, v.cmd);   // zeroes feet_air_time in HBM
#pragma unroll
        for (int f = 0; f < 4; ++f) sfat[tid][f] = 0.f;
        for (int c = 0; c < 24; ++c) srow[tid][c] = B.dof_state[(int64_t)e * 24 + c];  // post-reset rows
      }
      sbase[tid][0] = v.blv.x; sbase[tid][1] = v.blv.y; sbase[tid][2] = v.blv.z;
      sbase[tid][3] = v.bav.x; sbase[tid][4] = v.bav.y; sbase[tid][5] = v.bav.z;
      sbase[tid][6] = v.pg.x; sbase[tid][7] = v.pg.y; sbase[tid][8] = v.pg.z;
#pragma unroll
      for (int k = 0; k < 4; ++k) sbase[tid][9 + k] = v.cmd[k];
      sbase[tid][13] = v.reset ? rs[2] : rs0[2];   // post-reset root z
      for (int k = 0; k < 4; ++k) cmd_g[k] = v.cmd[k];
      if (P->curriculum) part[tid][T + 1] = (float)B.terrain_levels[e];
      float* o3 = B.base_lin_vel + (int64_t)e * 3;
      o3[0] = v.blv.x; o3[1] = v.blv.y; o3[2] = v.blv.z;
      o3 = B.base_ang_vel + (int64_t)e * 3;
      o3[0] = v.bav.x; o3[1] = v.bav.y; o3[2] = v.bav.z;
      o3 = B.projected_gravity + (int64_t)e * 3;
      o3[0] = v.pg.x; o3[1] = v.pg.y; o3[2] = v.pg.z;
    }
  }
  LGX_CLK(2);
  block_partials(part, T, B.scratch + (int64_t)blk * LGX_PARTIAL_STRIDE);
  const bool finalize = take_last_ticket(B, nblocks);
  for (int idx = tid; idx < T * LGX_ENV_BLOCK; idx += ENV_THREADS) {   // staged rows back
    const int t = idx / LGX_ENV_BLOCK, le = idx - t * LGX_ENV_BLOCK;
    if (e0 + le < N) B.episode_sums[(int64_t)t * N + e0 + le] = ssum[t][le];
  }
  if (tid < LGX_ENV_BLOCK * 4 && e0 + (tid >> 2) < N)
    B.feet_air_time[(int64_t)(e0 + (tid >> 2)) * 4 + (tid & 3)] = sfat[tid >> 2][tid & 3];

  LGX_CLK(3);
  // ---- phase C: observations (:214-231) + noise + clip (:103-104); a lane owns 4 consecutive
  // entries of a row, whose noise is one Philox block (LGX_DRAW_NOISE is a multiple of 4)
  // Two branch-free loops (the index ranges of one wave's lanes used to diverge over the five
  // source cases): entries 0..47 read their source through a per-index LDS offset into the
  // env's staged rows, the height entries 48.. (quads 12..) come from the scan.
  const int nq = (nobs + 3) >> 2;
  const int nq0 = min(nq, 12);
  __shared__ int16_t src_off[48];   // entry i < 48 -> float offset: sbase row (< 16) or srow row (+ 16)
  if (tid < 48) {
    const int i = tid;
    src_off[i] = (int16_t)(i < 12 ? i : i < 24 ? 16 + 2 * (i - 12) : i < 36 ? 16 + 2 * (i - 24) + 1
                                                                           : 16 + 36 + LGX_MAX_BODIES * 3 + i - 36);
  }
  __syncthreads();
  const bool noise = P->add_noise != 0;
  const float clip = P->clip_obs;
  for (int idx = tid; idx < LGX_ENV_BLOCK * nq0; idx += ENV_THREADS) {
    const int le = idx / nq0, q = idx - le * nq0;
    const int e = e0 + le;
    if (e >= N) continue;
    float nz[4] = {0.5f, 0.5f, 0.5f, 0.5f};
    if (noise) D.quad(e, (LGX_DRAW_NOISE >> 2) + q, step, 0u, nz);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = 4 * q + u;
      if (i >= nobs) break;
      const int so = src_off[i];
      const float v = so < 16 ? sbase[le][so] : srow[le][so - 16];   // (reference order, :216-226)
      float o = (v - obs_sub[i]) * obs_mul[i];
      if (noise) o += (2.f * nz[u] - 1.f) * obs_nsc[i];
      B.obs[(int64_t)e * nobs + i] = clampf(o, -clip, clip);
    }
  }
  const int nqh = nq - nq0;   // height quads
#pragma unroll 2
  for (int idx = tid; idx < LGX_ENV_BLOCK * nqh; idx += ENV_THREADS) {
    const int le = idx / nqh, q = nq0 + (idx - le * nqh);
    const int e = e0 + le;
    if (e >= N) continue;
    float nz[4] = {0.5f, 0.5f, 0.5f, 0.5f};
    if (noise) D.quad(e, (LGX_DRAW_NOISE >> 2) + q, step, 0u, nz);
    const float z = sbase[le][13] - 0.5f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = 4 * q + u;
      if (i >= nobs) break;
      const float v = clampf(z - sheight[le][i - 48], -1.f, 1.f);
      float o = (v - obs_sub[i]) * obs_mul[i];
      if (noise) o += (2.f * nz[u] - 1.f) * obs_nsc[i];
      B.obs[(int64_t)e * nobs + i] = clampf(o, -clip, clip);
    }
  }
  LGX_CLK(4);
  // ---- last_* copies (:136-138), post-reset values
  for (int idx = tid; idx < LGX_ENV_BLOCK * 12; idx += ENV_THREADS) {
    int e = e0 + idx / 12, j = idx % 12;
    if (e >= N) break;
    B.last_actions[(int64_t)e * 12 + j] = srow[idx / 12][36 + LGX_MAX_BODIES * 3 + j];
    B.last_dof_vel[(int64_t)e * 12 + j] = srow[idx / 12][2 * j + 1];
  }
  if (tid < LGX_ENV_BLOCK && e0 + tid < N) {
    int e = e0 + tid;
    for (int i = 0; i < 6; ++i) B.last_root_vel[(int64_t)e * 6 + i] = B.root_states[(int64_t)e * 13 + 7 + i];
  }
  LGX_CLK(5);
  LGX_CLK_PRINT("post_physics", 6)
  if (finalize) {
    __syncthreads();
    extras_finalize_body(P, B, nblocks, 0, snapshot, ENV_THREADS);
  }
}

}  // namespace

__global__ void __launch_bounds__(ENV_THREADS)
lgx_post_physics_kernel(const lgx_env_params* __restrict__ P, lgx_buffers B, int64_t step, const float* draws,
                        float* snapshot) {
  post_physics_body(P, B, step, draws, blockIdx.x, gridDim.x, snapshot);
}

// post-physics and the Go1 actuator network in ONE launch: workgroups [0, nblocks) are the
// post-physics workgroups, the rest persistent actuator-net workgroups.  The actuator output is
// not read by the env step (go1.py:71-73), so the two are independent; sharing a launch lets the
// latency-bound env logic and the MFMA-bound network fill the CUs together without a second
// stream's event record / wait per step.
__global__ void __launch_bounds__(ENV_THREADS, 2)
lgx_post_physics_act_kernel(const lgx_env_params* __restrict__ P, lgx_buffers B, int64_t step, const float* draws,
                            float* snapshot, WsArgs wa, int32_t nblocks) {
  if ((int)blockIdx.x < nblocks) post_physics_body(P, B, step, draws, blockIdx.x, nblocks, snapshot);
  else actuator_ws_body(wa, blockIdx.x - nblocks, gridDim.x - nblocks);
}

// reset_idx on an explicit env list (BaseTask.reset, base_task.py:111-115)
__global__ void __launch_bounds__(LGX_ENV_BLOCK)
lgx_reset_idx_kernel(const lgx_env_params* __restrict__ P, lgx_buffers B, const int32_t* ids, int32_t n, int64_t step,
                     int32_t init_done, const float* draws) {
  const int N = P->num_envs;
  const int T = P->num_terms + (P->termination_slot >= 0 ? 1 : 0);
  const Draws D{P, draws, LGX_DRAW_NOISE + P->num_obs};
  __shared__ float part[LGX_ENV_BLOCK][LGX_PARTIAL_STRIDE];
  int tid = threadIdx.x;
  int k = blockIdx.x * LGX_ENV_BLOCK + tid;
  for (int t = 0; t < LGX_PARTIAL_STRIDE; ++t) part[tid][t] = 0.f;
  if (k < n) {
    int e = ids[k];
    float cmd[4];
    for (int c = 0; c < 4; ++c) cmd[c] = B.commands[(int64_t)e * 4 + c];
    for (int t = 0; t < T; ++t) {
      part[tid][t] = B.episode_sums[(int64_t)t * N + e];
      B.episode_sums[(int64_t)t * N + e] = 0.f;
    }
    part[tid][T] = 1.f;
    reset_env(P, B, D, e, step, 1u, init_done != 0, cmd);
    for (int c = 0; c < 4; ++c) B.commands[(int64_t)e * 4 + c] = cmd[c];
  }
  block_partials(part, T, B.scratch + (int64_t)blockIdx.x * LGX_PARTIAL_STRIDE);
}

__global__ void __launch_bounds__(256)
lgx_extras_finalize_kernel(const lgx_env_params* __restrict__ P, lgx_buffers B, int32_t nblocks, int32_t level_scan,
                           float* __restrict__ snapshot) {
  extras_finalize_body(P, B, nblocks, level_scan, snapshot, 256);
}

int lgx_launch_post_physics(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int32_t num_obs,
                            int32_t n_term_rows, int32_t measure_heights, int64_t step, const float* draws,
                            float* extras_snapshot, hipStream_t stream) {
  (void)num_obs; (void)n_term_rows; (void)measure_heights;
  int blocks = (n_envs + LGX_ENV_BLOCK - 1) / LGX_ENV_BLOCK;
  LGX_LAUNCH(lgx_post_physics_kernel, dim3(blocks), dim3(ENV_THREADS), 0, stream, dp, b, step, draws,
             extras_snapshot);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_post_physics_act(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int64_t step,
                                const float* draws, float* extras_snapshot, const float* act_in, float* act_out,
                                int64_t act_rows, const float* act_w, const float* act_scale, hipStream_t stream) {
  static_assert(ENV_THREADS == 256, "the actuator-net workgroups are 256 threads");
  const int blocks = (n_envs + LGX_ENV_BLOCK - 1) / LGX_ENV_BLOCK;
  const int64_t tiles = (act_rows + WS_BM - 1) / WS_BM;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // one persistent actuator workgroup per CU next to the post-physics workgroups
  const int act_wgs = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, cus));
  WsArgs wa{act_in, act_out, act_rows, act_w, act_scale};
  LGX_LAUNCH(lgx_post_physics_act_kernel, dim3(blocks + act_wgs), dim3(ENV_THREADS), 0, stream, dp, b, step, draws,
             extras_snapshot, wa, blocks);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lgx_launch_reset_idx(const lgx_env_params* dp, const lgx_buffers& b, int32_t n_envs, int32_t n_term_rows,
                         const int32_t* ids, int32_t n, int64_t step, int32_t init_done, const float* draws,
                         float* extras_snapshot, hipStream_t stream) {
  (void)n_envs; (void)n_term_rows;
  if (n <= 0) return 0;
  int blocks = (n + LGX_ENV_BLOCK - 1) / LGX_ENV_BLOCK;
  hipLaunchKernelGGL(lgx_reset_idx_kernel, dim3(blocks), dim3(LGX_ENV_BLOCK), 0, stream, dp, b, ids, n, step,
                     init_done, draws);
  hipLaunchKernelGGL(lgx_extras_finalize_kernel, dim3(1), dim3(256), 0, stream, dp, b, blocks, 1, extras_snapshot);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
