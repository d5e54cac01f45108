// C-ABI implementation (include/lgx.h): validation, device-resident model/params, launch
// sequencing.  No host synchronisation in any step-path call; errors are reported through
// return codes + a thread-local message, never by exceptions across the ABI.
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "lgx_internal.h"

static thread_local std::string g_err;

static int fail(int code, const char* msg) {
  g_err = msg;
  return code;
}
static int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  g_err = buf;
  return LGX_EHIP;
}
int lgx_fail(int code, const char* msg) { return fail(code, msg); }
int lgx_hip_status(const char* what) { return hip_check(hipGetLastError(), what); }
static int launch_check(int rc, const char* what) {
  if (rc == 0) return 0;
  if (rc == -1) return fail(LGX_EINVAL, what);
  return hip_check(hipGetLastError(), what);
}

struct lgx_sim {
  int device;
  bool dense;             // physics on lgx_physics_dense_kernel (leg_dof 6 / LGX_PHYS_DENSE=1)
  int pp;                 // lanes per leg of the arrowhead physics kernel (lgx_physics_pp at create)
  int act_mode;           // where the Go1 actuator net runs (LGX_ACT_OVERLAP at create)
  int32_t num_points;     // contact candidates of the model (the dense kernel's LDS sizing)
  lgx_env_params params;  // host copy
  lgx_buffers bufs;
  lgx_dev_model* d_model;
  lgx_env_params* d_params;
  const float* draws;
  float* extras_snapshot;  // lgx_rebind_extras (NULL: no per-call copy)
  // Go1 actuator net off the critical path: its output (dVel) is not read by the step
  // (go1.py:71-73), so it runs on an auxiliary stream concurrently with post-physics and the
  // next policy forward; the next physics launch (which rewrites model_ins) waits for it.
  hipStream_t aux;
  hipEvent_t aux_in, aux_done;  // physics done (aux waits) / actuator done (main waits)
  bool aux_pending;
  int32_t n_term_rows;
  int32_t profiling;     // 0 = off, k = time every k-th lgx_step
  int64_t prof_calls;
  std::vector<hipEvent_t> ev[3];  // (start, stop) pairs per kernel class
  std::vector<hipEvent_t> pool;
};

static hipEvent_t take_event(lgx_sim* s) {
  if (!s->pool.empty()) { hipEvent_t e = s->pool.back(); s->pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  // no system-scope fences: the timestamps are only read back through hipEventElapsedTime
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}
thread_local lgx_timing_slot lgx_timing;

// arm the kernel-tight event pair for the next launch of kernel class `cls` (see LGX_LAUNCH)
static void arm(lgx_sim* s, int cls, bool sample) {
  lgx_timing = lgx_timing_slot{};
  if (!sample) return;
  hipEvent_t e0 = take_event(s), e1 = take_event(s);
  if (!e0 || !e1) return;
  s->ev[cls].push_back(e0);
  s->ev[cls].push_back(e1);
  lgx_timing = lgx_timing_slot{e0, e1};
}

extern "C" {

const char* lgx_last_error(void) { return g_err.c_str(); }
int lgx_version(void) { return 1; }
int32_t lgx_physics_lane_split(int32_t num_envs) { return num_envs > 0 ? lgx_physics_pp(num_envs) : LGX_EINVAL; }

void lgx_struct_sizes(int64_t out[12]) {
  out[0] = (int64_t)sizeof(lgx_model);
  out[1] = (int64_t)sizeof(lgx_env_params);
  out[2] = (int64_t)sizeof(lgx_buffers);
  out[3] = (int64_t)sizeof(lgx_mlp_desc);
  out[4] = (int64_t)sizeof(lgx_ppo_loss_args);
  out[5] = (int64_t)sizeof(lgx_reduce_job);
  out[6] = (int64_t)sizeof(lgx_ppo_act_args);
  out[7] = (int64_t)sizeof(lgx_ppo_store_args);
  out[8] = (int64_t)sizeof(lgx_gemm_args);
  out[9] = (int64_t)sizeof(lgx_copy2d_job);
  out[10] = (int64_t)sizeof(lgx_gemm_tn_args);
  out[11] = (int64_t)sizeof(lgx_mlp_x3_desc);
}

int64_t lgx_scratch_floats(int32_t num_envs, int32_t num_terms) {
  (void)num_terms;
  int64_t blocks = (num_envs + LGX_ENV_BLOCK - 1) / LGX_ENV_BLOCK;
  return blocks * LGX_PARTIAL_STRIDE + 64;
}

int lgx_sim_create(const lgx_model* model, const lgx_env_params* params, const lgx_buffers* bufs, int device,
                   lgx_sim** out) {
  if (!model || !params || !bufs || !out) return fail(LGX_EINVAL, "lgx_sim_create: null argument");
  if (params->num_envs <= 0) return fail(LGX_EINVAL, "lgx_sim_create: num_envs must be > 0");
  if (params->num_obs <= 0 || params->num_obs > LGX_MAX_OBS) return fail(LGX_EINVAL, "lgx_sim_create: bad num_obs");
  if (params->measure_heights && (params->num_height_points <= 0 || params->num_height_points > LGX_MAX_HEIGHT_POINTS ||
                                  48 + params->num_height_points != params->num_obs))
    return fail(LGX_EINVAL, "lgx_sim_create: num_obs must be 48 + num_height_points when measuring heights");
  if (!params->measure_heights && params->num_obs != 48)
    return fail(LGX_EINVAL, "lgx_sim_create: num_obs must be 48 without height measurements");
  if (params->num_terms < 0 || params->num_terms + 1 > LGX_MAX_TERMS) return fail(LGX_EINVAL, "lgx_sim_create: too many reward terms");
  if (params->decimation <= 0) return fail(LGX_EINVAL, "lgx_sim_create: decimation must be > 0");
  if (params->resample_interval <= 0) return fail(LGX_EINVAL, "lgx_sim_create: resample_interval must be > 0");
  if (params->push_robots && params->push_interval <= 0) return fail(LGX_EINVAL, "lgx_sim_create: push_interval must be > 0");
  if (model->num_points < 0 || model->num_points > LGX_MAX_POINTS) return fail(LGX_EINVAL, "lgx_sim_create: bad num_points");
  if (params->terrain_kind != 0 && (!bufs->height_samples || bufs->hf_rows < 2 || bufs->hf_cols < 2))
    return fail(LGX_EINVAL, "lgx_sim_create: terrain requires height_samples");
  const void* required[] = {bufs->root_states, bufs->dof_state, bufs->dof_targets, bufs->torques, bufs->contact_forces,
                            bufs->actions, bufs->last_actions, bufs->last_dof_vel, bufs->last_root_vel, bufs->commands,
                            bufs->base_lin_vel, bufs->base_ang_vel, bufs->projected_gravity, bufs->feet_air_time,
                            bufs->obs, bufs->rew, bufs->reset, bufs->time_out, bufs->episode_length,
                            bufs->episode_sums, bufs->env_origins, bufs->body_mass_scale, bufs->extras,
                            bufs->extras_time_outs, bufs->scratch};
  for (const void* p : required)
    if (!p) return fail(LGX_EINVAL, "lgx_sim_create: a required buffer is null");
  if (params->measure_heights && !bufs->measured_heights) return fail(LGX_EINVAL, "lgx_sim_create: measured_heights is null");
  if (params->use_actuator_history && (!bufs->act_hist || !bufs->model_ins))
    return fail(LGX_EINVAL, "lgx_sim_create: actuator history buffers are null");
  if (params->control_type < LGX_CTRL_POS_DRIVE || params->control_type > LGX_CTRL_SEA)
    return fail(LGX_EINVAL, "lgx_sim_create: bad control_type");
  if (params->control_type == LGX_CTRL_SEA && (!bufs->sea_w || !bufs->sea_h || !bufs->sea_c))
    return fail(LGX_EINVAL, "lgx_sim_create: LGX_CTRL_SEA needs sea_w / sea_h / sea_c");
  if (params->curriculum && (!bufs->terrain_levels || !bufs->terrain_types || !bufs->terrain_origins))
    return fail(LGX_EINVAL, "lgx_sim_create: curriculum buffers are null");

  // the dense joint-space kernel for the 2 x 6 biped (and, as an A/B and cross-check path, for any
  // robot with LGX_PHYS_DENSE=1); the arrowhead kernel for the 4 x 3 quadrupeds
  const int leg_dof = model->leg_dof == 0 ? 3 : model->leg_dof;
  if (leg_dof != 3 && leg_dof != 6) return fail(LGX_EINVAL, "lgx_sim_create: leg_dof must be 3 or 6");
  const char* force_dense = getenv("LGX_PHYS_DENSE");
  const bool dense = leg_dof == 6 || (force_dense && atoi(force_dense) == 1);
  if (dense && (params->control_type == LGX_CTRL_SEA || params->use_actuator_history))
    return fail(LGX_EINVAL, "lgx_sim_create: the dense physics kernel has no SEA / actuator-history drive inputs");
  // every contact candidate's dynamic body and reporting body index into fixed tables (LDS in both
  // physics kernels): checked for every point, whichever kernel runs
  for (int i = 0; i < model->num_points; ++i) {
    if (model->point_dyn[i] < 0 || model->point_dyn[i] >= LGX_NUM_DYN)
      return fail(LGX_EINVAL, "lgx_sim_create: bad point_dyn");
    if (model->point_report[i] < 0 || model->point_report[i] >= LGX_MAX_BODIES)
      return fail(LGX_EINVAL, "lgx_sim_create: bad point_report");
  }
  // per-lane contact candidate tables: leg points to their leg's lane, base points round-robin
  lgx_dev_model dm;
  memset(&dm, 0, sizeof dm);
  dm.m = *model;
  dm.m.leg_dof = leg_dof;
  int rr = 0;
  for (int i = 0; i < (dense ? 0 : model->num_points); ++i) {
    int d = model->point_dyn[i];
    int rep = model->point_report[i];
    if (d < 0 || d >= LGX_NUM_DYN) return fail(LGX_EINVAL, "lgx_sim_create: bad point_dyn");
    int lane;
    if (d == 0) {
      if (rep != 0) return fail(LGX_EINVAL, "lgx_sim_create: base points must report on body 0");
      lane = rr++ & 3;
    } else {
      lane = (d - 1) / 3;
      if (rep < 1 + 4 * lane || rep > 4 + 4 * lane) return fail(LGX_EINVAL, "lgx_sim_create: leg point reports on a foreign body");
    }
    if (dm.lane_npts[lane] >= LGX_MAX_LANE_PTS) return fail(LGX_EINVAL, "lgx_sim_create: too many contact points per leg");
    dm.lane_pts[lane][dm.lane_npts[lane]++] = i;
  }
  for (int l = 0; l < 4; ++l) dm.max_lane_npts = dm.lane_npts[l] > dm.max_lane_npts ? dm.lane_npts[l] : dm.max_lane_npts;
  dm.joint_rot_eye = 1;
  for (int j = 0; j < LGX_NUM_DOF; ++j)
    for (int i = 0; i < 9; ++i)
      if (model->joint_rot[j][i] != (i % 4 == 0 ? 1.f : 0.f)) dm.joint_rot_eye = 0;

  int rc = hip_check(hipSetDevice(device), "hipSetDevice");
  if (rc) return rc;
  lgx_sim* s = new (std::nothrow) lgx_sim();
  if (!s) return fail(LGX_ENOMEM, "lgx_sim_create: out of host memory");
  s->device = device;
  s->dense = dense;
  s->pp = lgx_physics_pp(params->num_envs);
  // where the Go1 actuator net runs (LGX_ACT_OVERLAP, read here once): 2 (default) = on workgroups
  // of its own inside the post-physics launch, 1 = its own launch on an auxiliary stream, 0 = its
  // own launch on the caller's stream (the PMC passes that measure it alone)
  const char* am = getenv("LGX_ACT_OVERLAP");
  s->act_mode = am && *am ? atoi(am) : 2;
  if (s->act_mode < 0 || s->act_mode > 2 || (am && *am && (am[0] < '0' || am[0] > '2' || am[1]))) {
    delete s;
    return fail(LGX_EINVAL, "lgx_sim_create: LGX_ACT_OVERLAP must be 0, 1 or 2");
  }
  s->num_points = model->num_points;
  s->params = *params;
  s->bufs = *bufs;
  s->draws = nullptr;
  s->extras_snapshot = nullptr;
  s->aux = nullptr;
  s->aux_in = s->aux_done = nullptr;
  s->aux_pending = false;
  s->profiling = 0;
  s->prof_calls = 0;
  s->n_term_rows = params->num_terms + (params->termination_slot >= 0 ? 1 : 0);
  if ((rc = hip_check(hipMalloc(&s->d_model, sizeof(lgx_dev_model)), "hipMalloc(model)"))) { delete s; return rc; }
  if ((rc = hip_check(hipMalloc(&s->d_params, sizeof(lgx_env_params)), "hipMalloc(params)"))) {
    (void)hipFree(s->d_model); delete s; return rc;
  }
  rc = hip_check(hipMemcpy(s->d_model, &dm, sizeof dm, hipMemcpyHostToDevice), "hipMemcpy(model)");
  if (!rc) rc = hip_check(hipMemcpy(s->d_params, params, sizeof *params, hipMemcpyHostToDevice), "hipMemcpy(params)");
  // the post-physics completion ticket (after the block partials in scratch) starts at zero
  if (!rc) {
    const int64_t blocks = (params->num_envs + LGX_ENV_BLOCK - 1) / LGX_ENV_BLOCK;
    rc = hip_check(hipMemset(bufs->scratch + blocks * LGX_PARTIAL_STRIDE, 0, sizeof(unsigned int)), "hipMemset(ticket)");
  }
  if (rc) { (void)hipFree(s->d_model); (void)hipFree(s->d_params); delete s; return rc; }
  *out = s;
  return 0;
}

int lgx_sim_destroy(lgx_sim* s) {
  if (!s) return 0;
  if (s->aux) {
    (void)hipStreamSynchronize(s->aux);
    (void)hipStreamDestroy(s->aux);
    (void)hipEventDestroy(s->aux_in);
    (void)hipEventDestroy(s->aux_done);
  }
  for (auto& v : s->ev) for (hipEvent_t e : v) (void)hipEventDestroy(e);
  for (hipEvent_t e : s->pool) (void)hipEventDestroy(e);
  (void)hipFree(s->d_model);
  (void)hipFree(s->d_params);
  delete s;
  return 0;
}

int lgx_sim_buffer(lgx_sim* s, int32_t id, void** ptr, int64_t shape[4], int32_t* ndim, int32_t* dtype) {
  if (!s || !ptr || !shape || !ndim || !dtype) return fail(LGX_EINVAL, "lgx_sim_buffer: null argument");
  const int64_t N = s->params.num_envs;
  const lgx_buffers& b = s->bufs;
  struct Entry { void* p; int nd; int64_t d[3]; int dt; };
  Entry e;
  switch (id) {
    case LGX_BUF_ROOT_STATES: e = {b.root_states, 2, {N, 13}, LGX_F32}; break;
    case LGX_BUF_DOF_STATE: e = {b.dof_state, 3, {N, LGX_NUM_DOF, 2}, LGX_F32}; break;
    case LGX_BUF_DOF_TARGETS: e = {b.dof_targets, 2, {N, LGX_NUM_DOF}, LGX_F32}; break;
    case LGX_BUF_TORQUES: e = {b.torques, 2, {N, LGX_NUM_DOF}, LGX_F32}; break;
    case LGX_BUF_CONTACT_FORCES: e = {b.contact_forces, 3, {N, LGX_MAX_BODIES, 3}, LGX_F32}; break;
    case LGX_BUF_ACTIONS: e = {b.actions, 2, {N, LGX_NUM_DOF}, LGX_F32}; break;
    case LGX_BUF_LAST_ACTIONS: e = {b.last_actions, 2, {N, LGX_NUM_DOF}, LGX_F32}; break;
    case LGX_BUF_LAST_DOF_VEL: e = {b.last_dof_vel, 2, {N, LGX_NUM_DOF}, LGX_F32}; break;
    case LGX_BUF_LAST_ROOT_VEL: e = {b.last_root_vel, 2, {N, 6}, LGX_F32}; break;
    case LGX_BUF_COMMANDS: e = {b.commands, 2, {N, 4}, LGX_F32}; break;
    case LGX_BUF_BASE_LIN_VEL: e = {b.base_lin_vel, 2, {N, 3}, LGX_F32}; break;
    case LGX_BUF_BASE_ANG_VEL: e = {b.base_ang_vel, 2, {N, 3}, LGX_F32}; break;
    case LGX_BUF_PROJECTED_GRAVITY: e = {b.projected_gravity, 2, {N, 3}, LGX_F32}; break;
    case LGX_BUF_FEET_AIR_TIME: e = {b.feet_air_time, 2, {N, 4}, LGX_F32}; break;
    case LGX_BUF_OBS: e = {b.obs, 2, {N, s->params.num_obs}, LGX_F32}; break;
    case LGX_BUF_REW: e = {b.rew, 1, {N}, LGX_F32}; break;
    case LGX_BUF_RESET: e = {b.reset, 1, {N}, LGX_U8}; break;
    case LGX_BUF_TIME_OUT: e = {b.time_out, 1, {N}, LGX_U8}; break;
    case LGX_BUF_EPISODE_LENGTH: e = {b.episode_length, 1, {N}, LGX_I64}; break;
    case LGX_BUF_EPISODE_SUMS: e = {b.episode_sums, 2, {s->n_term_rows, N}, LGX_F32}; break;
    case LGX_BUF_MEASURED_HEIGHTS: e = {b.measured_heights, 2, {N, s->params.num_height_points}, LGX_F32}; break;
    case LGX_BUF_ENV_ORIGINS: e = {b.env_origins, 2, {N, 3}, LGX_F32}; break;
    case LGX_BUF_TERRAIN_LEVELS: e = {b.terrain_levels, 1, {N}, LGX_I64}; break;
    case LGX_BUF_TERRAIN_TYPES: e = {b.terrain_types, 1, {N}, LGX_I64}; break;
    case LGX_BUF_EXTRAS: e = {b.extras, 1, {s->n_term_rows + 2}, LGX_F32}; break;
    default: return fail(LGX_EINVAL, "lgx_sim_buffer: unknown buffer id");
  }
  *ptr = e.p;
  *ndim = e.nd;
  *dtype = e.dt;
  for (int i = 0; i < 4; ++i) shape[i] = i < e.nd ? e.d[i] : 1;
  return 0;
}

int lgx_set_draws(lgx_sim* s, const float* draws) {
  if (!s) return fail(LGX_EINVAL, "lgx_set_draws: null sim");
  s->draws = draws;
  return 0;
}

int lgx_rebind_obs(lgx_sim* s, float* obs) {
  if (!s || !obs) return fail(LGX_EINVAL, "lgx_rebind_obs: null argument");
  s->bufs.obs = obs;
  return 0;
}

int lgx_rebind_extras(lgx_sim* s, float* snapshot) {
  if (!s) return fail(LGX_EINVAL, "lgx_rebind_extras: null sim");
  s->extras_snapshot = snapshot;
  return 0;
}

// make `st` wait for the outstanding auxiliary-stream work (the actuator net of the last step)
static int join_aux(lgx_sim* s, hipStream_t st) {
  if (!s->aux_pending) return 0;
  return hip_check(hipStreamWaitEvent(st, s->aux_done, 0), "hipStreamWaitEvent(aux)");
}


int lgx_sync_aux(lgx_sim* s, void* stream) {
  if (!s) return fail(LGX_EINVAL, "lgx_sync_aux: null sim");
  return join_aux(s, (hipStream_t)stream);
}

// the physics launch of a sim: the arrowhead kernel, or the dense one (lgx_sim.dense)
static int physics(lgx_sim* s, int32_t nsub, int32_t from_actions, const float* actions, hipStream_t st, int32_t frozen) {
  return s->dense ? lgx_launch_physics_dense(s->d_model, s->d_params, s->bufs, s->params.num_envs, nsub, from_actions,
                                             actions, st, frozen, s->num_points)
                  : lgx_launch_physics(s->d_model, s->d_params, s->bufs, s->params.num_envs, nsub, from_actions, actions,
                                       st, frozen, s->pp);
}

int lgx_simulate(lgx_sim* s, int32_t n, void* stream) {
  if (!s || n < 0) return fail(LGX_EINVAL, "lgx_simulate: bad arguments");
  if (n == 0) return 0;
  if (int rc = join_aux(s, (hipStream_t)stream)) return rc;
  return launch_check(physics(s, n, 0, nullptr, (hipStream_t)stream, 0), "lgx_simulate: physics launch");
}

int lgx_drive_inputs(lgx_sim* s, const float* actions, void* stream) {
  if (!s) return fail(LGX_EINVAL, "lgx_drive_inputs: null sim");
  if (int rc = join_aux(s, (hipStream_t)stream)) return rc;   // the last actuator net still reads model_ins
  return launch_check(physics(s, s->params.decimation, 1, actions, (hipStream_t)stream, 1), "lgx_drive_inputs: launch");
}

int lgx_ground_contact(lgx_sim* s, const float* points, int32_t n, float* out, void* stream) {
  if (!s || n < 0 || (n > 0 && (!points || !out))) return fail(LGX_EINVAL, "lgx_ground_contact: bad arguments");
  return launch_check(lgx_launch_ground_contact(s->d_params, s->bufs, points, n, out, (hipStream_t)stream),
                      "lgx_ground_contact: launch");
}

int lgx_post_physics(lgx_sim* s, int64_t step, void* stream) {
  if (!s) return fail(LGX_EINVAL, "lgx_post_physics: null sim");
  return launch_check(lgx_launch_post_physics(s->d_params, s->bufs, s->params.num_envs, s->params.num_obs, s->n_term_rows,
                                              s->params.measure_heights, step, s->draws, s->extras_snapshot,
                                              (hipStream_t)stream),
                      "lgx_post_physics: launch");
}

static int post_physics_fused(lgx_sim* s, int64_t step, hipStream_t st, bool sample);

int lgx_step(lgx_sim* s, int64_t step, void* stream) { return lgx_step_from(s, nullptr, step, stream); }

int lgx_step_from(lgx_sim* s, const float* actions, int64_t step, void* stream) {
  if (!s) return fail(LGX_EINVAL, "lgx_step: null sim");
  hipStream_t st = (hipStream_t)stream;
  const lgx_env_params& p = s->params;
  const bool sample = s->profiling > 0 && (s->prof_calls++ % s->profiling) == 0;
  // action clipping is fused into the physics kernel's action load (raw actions from `actions`
  // or, when NULL, from the bound actions buffer; the clipped copy lands in the bound buffer)
  int rc = join_aux(s, st);  // the last actuator net still reads model_ins
  if (rc) return rc;
  arm(s, 0, sample);
  rc = launch_check(physics(s, p.decimation, 1, actions, st, 0), "lgx_step: physics launch");
  if (rc) return rc;
  return post_physics_fused(s, step, st, sample);
}

// the second launch(es) of lgx_step_from: post-physics with the Go1 actuator net over this step's
// model_ins - one launch by default (act_mode 2), or the actuator on its own launch / stream
static int post_physics_fused(lgx_sim* s, int64_t step, hipStream_t st, bool sample) {
  const lgx_env_params& p = s->params;
  int rc = 0;
  const bool act_net = p.use_actuator_history && s->bufs.act_net_w && s->bufs.act_dvel;
  const int mode = s->act_mode;
  if (act_net && mode == 2) {
    // UniNet on every (substep, env, leg) row of this step's model_ins, inside the post-physics
    // launch (the next physics launch, stream-ordered after it, rewrites model_ins)
    arm(s, 2, sample);
    rc = launch_check(lgx_launch_post_physics_act(s->d_params, s->bufs, p.num_envs, step, s->draws, s->extras_snapshot,
                                                  s->bufs.model_ins, s->bufs.act_dvel,
                                                  (int64_t)p.decimation * p.num_envs * 4, s->bufs.act_net_w,
                                                  s->bufs.act_net_scale, st),
                      "lgx_step: post-physics + actuator launch");
    lgx_timing = lgx_timing_slot{};
    return rc;
  }
  if (act_net) {
    // UniNet on every (substep, env, leg) row of this step's model_ins; result = dVel
    hipStream_t ast = st;
    if (mode == 1) {
      if (!s->aux) {
        rc = hip_check(hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking), "hipStreamCreate(aux)");
        if (!rc) rc = hip_check(hipEventCreateWithFlags(&s->aux_in, hipEventDisableTiming), "hipEventCreate(aux)");
        if (!rc) rc = hip_check(hipEventCreateWithFlags(&s->aux_done, hipEventDisableTiming), "hipEventCreate(aux)");
        if (rc) return rc;
      }
      rc = hip_check(hipEventRecord(s->aux_in, st), "hipEventRecord(aux_in)");
      if (!rc) rc = hip_check(hipStreamWaitEvent(s->aux, s->aux_in, 0), "hipStreamWaitEvent(aux_in)");
      if (rc) return rc;
      ast = s->aux;
    }
    arm(s, 1, sample);
    rc = launch_check(lgx_launch_actuator_mlp(s->bufs.model_ins, s->bufs.act_dvel, (int64_t)p.decimation * p.num_envs * 4,
                                              s->bufs.act_net_w, s->bufs.act_net_scale, ast, ast != st ? 1 : 2),
                      "lgx_step: actuator mlp launch");
    if (rc) return rc;
    if (ast != st) {
      rc = hip_check(hipEventRecord(s->aux_done, ast), "hipEventRecord(aux_done)");
      if (rc) return rc;
      s->aux_pending = true;
    }
  }
  arm(s, 2, sample);
  rc = lgx_post_physics(s, step, st);
  lgx_timing = lgx_timing_slot{};
  return rc;
}

int lgx_post_physics_fused(lgx_sim* s, int64_t step, void* stream) {
  if (!s) return fail(LGX_EINVAL, "lgx_post_physics_fused: null sim");
  return post_physics_fused(s, step, (hipStream_t)stream, false);
}

int lgx_profile_enable(lgx_sim* s, int32_t on) {
  if (!s) return fail(LGX_EINVAL, "lgx_profile_enable: null sim");
  s->profiling = on > 0 ? on : 0;
  s->prof_calls = 0;
  return 0;
}

int lgx_profile_collect(lgx_sim* s, double* ms, int64_t* count) {
  if (!s || !ms || !count) return fail(LGX_EINVAL, "lgx_profile_collect: null argument");
  for (int c = 0; c < 3; ++c) {
    double tot = 0.0;
    int64_t n = 0;
    auto& v = s->ev[c];
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
      int rc = hip_check(hipEventSynchronize(v[i + 1]), "hipEventSynchronize");
      if (rc) return rc;
      float t = 0.f;
      rc = hip_check(hipEventElapsedTime(&t, v[i], v[i + 1]), "hipEventElapsedTime");
      if (rc) return rc;
      tot += t;
      ++n;
    }
    for (hipEvent_t e : v) s->pool.push_back(e);
    v.clear();
    ms[c] = tot;
    count[c] = n;
  }
  return 0;
}

int lgx_reset_idx(lgx_sim* s, const int32_t* env_ids, int32_t n, int64_t step, int32_t init_done, void* stream) {
  if (!s || n < 0 || (n > 0 && !env_ids)) return fail(LGX_EINVAL, "lgx_reset_idx: bad arguments");
  if (n > s->params.num_envs) return fail(LGX_EINVAL, "lgx_reset_idx: more ids than envs");
  return launch_check(lgx_launch_reset_idx(s->d_params, s->bufs, s->params.num_envs, s->n_term_rows, env_ids, n, step,
                                           init_done, s->draws, s->extras_snapshot, (hipStream_t)stream),
                      "lgx_reset_idx: launch");
}

int lgx_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale, void* stream) {
  if (!in || !out || !w || rows < 0) return fail(LGX_EINVAL, "lgx_actuator_mlp: bad arguments");
  return launch_check(lgx_launch_actuator_mlp(in, out, rows, w, out_scale, (hipStream_t)stream), "lgx_actuator_mlp: launch");
}

int lgx_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w, void* stream) {
  if (!x || !h || !c || !tau || !w || m < 0) return fail(LGX_EINVAL, "lgx_actuator_lstm: bad arguments");
  return launch_check(lgx_launch_actuator_lstm(x, h, c, tau, m, w, (hipStream_t)stream), "lgx_actuator_lstm: launch");
}

int lgx_mlp_forward(const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims, const float* const* weights,
                    const float* const* biases, int32_t act, void* stream) {
  if (!x || !y || !dims || !weights || !biases || rows < 0) return fail(LGX_EINVAL, "lgx_mlp_forward: bad arguments");
  return launch_check(lgx_launch_mlp_forward(x, y, rows, nl, dims, weights, biases, act, (hipStream_t)stream),
                      "lgx_mlp_forward: launch (widths must be 1..512, layers 1..6)");
}

int lgx_mlp_forward_batch(const lgx_mlp_desc* descs, int32_t count, void* stream) {
  if (!descs) return fail(LGX_EINVAL, "lgx_mlp_forward_batch: null descs");
  return launch_check(lgx_launch_mlp_forward2(descs, count, (hipStream_t)stream),
                      "lgx_mlp_forward_batch: launch (count 1..2, widths 1..512, layers 1..6)");
}

int lgx_gae(const float* rewards, const float* values, const uint8_t* dones, const float* last_values, float* returns,
            float* advantages, int32_t T, int32_t N, float gamma, float lam, void* stream) {
  if (!rewards || !values || !dones || !last_values || !returns || !advantages)
    return fail(LGX_EINVAL, "lgx_gae: null argument");
  return launch_check(lgx_launch_gae(rewards, values, dones, last_values, returns, advantages, T, N, gamma, lam,
                                     (hipStream_t)stream),
                      "lgx_gae: launch (T, N must be > 0)");
}

int64_t lgx_gae_norm_scratch(int32_t N) { return N > 0 ? 3 * (int64_t)((N + 255) / 256) : -1; }

int lgx_gae_norm(const float* rewards, const float* values, const uint8_t* dones, const float* last_values,
                 float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam, double* scratch,
                 void* stream) {
  if (!rewards || !values || !dones || !last_values || !returns || !advantages || !scratch)
    return fail(LGX_EINVAL, "lgx_gae_norm: null argument");
  return launch_check(lgx_launch_gae_norm(rewards, values, dones, last_values, returns, advantages, T, N, gamma, lam,
                                          scratch, (hipStream_t)stream),
                      "lgx_gae_norm: launch (T, N must be > 0)");
}

int lgx_gae_parts(const float* rewards, const float* values, const uint8_t* dones, const float* last_values,
                  float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam, double* parts,
                  void* stream) {
  if (!rewards || !values || !dones || !last_values || !returns || !advantages || !parts)
    return fail(LGX_EINVAL, "lgx_gae_parts: null argument");
  return launch_check(lgx_launch_gae_parts(rewards, values, dones, last_values, returns, advantages, T, N, gamma, lam,
                                           parts, (hipStream_t)stream),
                      "lgx_gae_parts: launch (T, N must be > 0)");
}

int lgx_adv_norm(float* advantages, int64_t n, const double* parts, int32_t nparts, void* stream) {
  if (!advantages || !parts) return fail(LGX_EINVAL, "lgx_adv_norm: null argument");
  return launch_check(lgx_launch_adv_norm(advantages, n, parts, nparts, (hipStream_t)stream),
                      "lgx_adv_norm: launch (n, nparts must be > 0)");
}

}  // extern "C"

// ---- device-scope cross-stream events (lgx.h: lgx_event_create)
extern "C" int lgx_event_create(void** ev) {
  if (!ev) return lgx_fail(LGX_EINVAL, "lgx_event_create: null out pointer");
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
    return lgx_fail(LGX_EHIP, "lgx_event_create: hipEventCreateWithFlags failed");
  *ev = reinterpret_cast<void*>(e);
  return LGX_OK;
}
extern "C" int lgx_event_destroy(void* ev) {
  if (!ev) return LGX_OK;
  return hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)) == hipSuccess ? LGX_OK
                                                                         : lgx_fail(LGX_EHIP, "lgx_event_destroy failed");
}
extern "C" int lgx_event_record(void* ev, void* stream) {
  if (!ev) return lgx_fail(LGX_EINVAL, "lgx_event_record: null event");
  return hipEventRecord(reinterpret_cast<hipEvent_t>(ev), reinterpret_cast<hipStream_t>(stream)) == hipSuccess
             ? LGX_OK
             : lgx_fail(LGX_EHIP, "lgx_event_record: hipEventRecord failed");
}
// Bind a device event to the completion of the NEXT lgx launch on this thread (its dispatch records
// it: hipExtLaunchKernelGGL's stop event - no separate marker packet on the producer stream, whose
// processing leaves the stream idle ~5 us between two kernels); lgx_launch_bind_pending: 1 when
// no launch has taken the event since (the caller then records it itself), and disarms.
extern "C" int lgx_launch_bind_event(void* ev) {
  if (!ev) return lgx_fail(LGX_EINVAL, "lgx_launch_bind_event: null event");
  lgx_timing = lgx_timing_slot{nullptr, reinterpret_cast<hipEvent_t>(ev)};
  return LGX_OK;
}
extern "C" int lgx_launch_bind_pending(void) {
  const int pending = (lgx_timing.start || lgx_timing.stop) ? 1 : 0;
  lgx_timing = lgx_timing_slot{};
  return pending;
}
extern "C" int lgx_stream_wait_event(void* stream, void* ev) {
  if (!ev) return lgx_fail(LGX_EINVAL, "lgx_stream_wait_event: null event");
  return hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<hipEvent_t>(ev), 0) == hipSuccess
             ? LGX_OK
             : lgx_fail(LGX_EHIP, "lgx_stream_wait_event: hipStreamWaitEvent failed");
}
