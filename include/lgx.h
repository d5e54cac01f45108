/*
 * lgx.h — C-ABI of the MI355X-native legged-robot rollout engine (liblgx.so).
 *
 * This is the drop-in boundary that replaces the Isaac Gym tensor API used by the
 * reference's LeggedRobot.  Each entry point cites the reference
 * call(s) it replaces.  Conventions:
 *   - plain C types only; every buffer is a *device* pointer owned by the caller
 *     (the Python host allocates them as torch tensors and binds them once with
 *     lgx_sim_create); the library owns only its constant tables and scratch;
 *   - every call returns 0 on success and a negative LGX_E* code on failure;
 *     lgx_last_error() returns a thread-local message; no C++ exception crosses the ABI;
 *   - every launch is stream-ordered on the `stream` argument (a hipStream_t), no
 *     host synchronisation happens inside any call (graph-capturable);
 *   - one lgx_sim per GPU / rank; an instance is not thread-safe.
 *
 * Layouts (row-major, N = num_envs, units SI, quaternions xyzw as in the reference):
 *   root_states [N,13]   pos3 quat4 linvel3 angvel3, world frame   (legged_robot.py:518)
 *   dof_state   [N,12,2] (pos, vel) interleaved per DOF             (legged_robot.py:519-521)
 *   contact_forces [N,B,3] net ground contact force per body         (legged_robot.py:524)
 *   torques     [N,12]   applied joint drive torque                  (legged_robot.py:536)
 */
#ifndef LGX_H
#define LGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LGX_NUM_LEGS 4
#define LGX_NUM_DOF 12
#define LGX_NUM_DYN 13          /* base + 4 legs x (hip, thigh, shank+foot) */
#define LGX_MAX_BODIES 17       /* reporting bodies in the contact-force tensor */
#define LGX_MAX_POINTS 128      /* contact primitives (sphere centres / box corners) */
#define LGX_MAX_OBS 256
#define LGX_MAX_HEIGHT_POINTS 192
#define LGX_MAX_TERMS 24

/* error codes */
#define LGX_OK 0
#define LGX_EINVAL -1
#define LGX_EHIP -2
#define LGX_ENOMEM -3

/* reward term ids: one per reference `_reward_<name>` (legged_robot.py:857-966) */
enum lgx_reward_term {
  LGX_R_LIN_VEL_Z = 0, LGX_R_ANG_VEL_XY, LGX_R_ORIENTATION, LGX_R_BASE_HEIGHT, LGX_R_TORQUES,
  LGX_R_ENERGY, LGX_R_DOF_VEL, LGX_R_DOF_ACC, LGX_R_ACTION_RATE, LGX_R_COLLISION,
  LGX_R_TERMINATION, LGX_R_DOF_POS_LIMITS, LGX_R_DOF_VEL_LIMITS, LGX_R_TORQUE_LIMITS,
  LGX_R_TRACKING_LIN_VEL, LGX_R_TRACKING_ANG_VEL, LGX_R_FEET_AIR_TIME, LGX_R_STUMBLE,
  LGX_R_STAND_STILL, LGX_R_FEET_CONTACT_FORCES, LGX_R_HIP_MOTION,
  LGX_R_NO_FLY,  /* Cassie: exactly one foot with F_z > 0.1 N (envs/cassie/cassie.py:42-46) */
  LGX_R_COUNT
};

/* control paths: position drive (the reference step path, legged_robot.py:93-96) or
 * the explicit-torque `_compute_torques` variants (legged_robot.py:370-392): the P / V / T laws of
 * LeggedRobot._compute_torques, or LGX_CTRL_SEA = ANYmal's override (anymal.py:71-78), the SEA
 * actuator-network LSTM as the torque source (lgx_buffers.sea_*), advanced once per substep */
enum lgx_control { LGX_CTRL_POS_DRIVE = 0, LGX_CTRL_P = 1, LGX_CTRL_V = 2, LGX_CTRL_T = 3, LGX_CTRL_SEA = 4 };

/* Per-env uniform draws: slot layout of one env's row (stride LGX_DRAW_NOISE + num_obs).
 * In production the draws come from an in-kernel Philox4x32-10 stream keyed by
 * (seed, env, step counter); for golden parity the caller injects them (lgx_set_draws). */
#define LGX_DRAW_CMD 0          /* 3: periodic command resample (legged_robot.py:342,360-365) */
#define LGX_DRAW_PUSH 3         /* 2: push velocity xy (legged_robot.py:440) */
#define LGX_DRAW_RESET_DOF 5    /* 12: dof factor U[0.5,1.5] (legged_robot.py:407) */
#define LGX_DRAW_RESET_XY 17    /* 2: origin offset U[-1,1] (legged_robot.py:425) */
#define LGX_DRAW_RESET_VEL 19   /* 6: root vel U[-.5,.5] (legged_robot.py:430) */
#define LGX_DRAW_RESET_CMD 25   /* 3: command resample on reset (legged_robot.py:173) */
#define LGX_DRAW_CURRIC 28      /* 1: randint level on curriculum wrap (legged_robot.py:461) */
#define LGX_DRAW_NOISE 32       /* num_obs: obs noise U[0,1) (legged_robot.py:231) */

typedef struct lgx_model {
  /* kinematic tree: 12 revolute joints in serial leg chains of leg_dof joints off the base (4 x 3:
   * the quadrupeds; 2 x 6: Cassie); joint j = leg_dof*leg + k moves dyn body 1 + j, its parent is
   * the base (k == 0) or dyn body j (k > 0).  Joint frame = parent frame * (rot, pos); child body
   * frame = joint frame * Rot(axis, q_j). */
  float joint_rot[LGX_NUM_DOF][9];
  float joint_pos[LGX_NUM_DOF][3];
  float joint_axis[LGX_NUM_DOF][3];
  float dof_lower[LGX_NUM_DOF];     /* hard limits (URDF); lower >= upper => unlimited */
  float dof_upper[LGX_NUM_DOF];
  float dof_vel_limit[LGX_NUM_DOF]; /* URDF velocity, PhysX maxJointVelocity */
  float dof_effort[LGX_NUM_DOF];    /* URDF effort = drive force limit */
  float kp[LGX_NUM_DOF];            /* drive stiffness (legged_robot.py:692-699) */
  float kd[LGX_NUM_DOF];            /* drive damping */
  /* dynamic bodies: nominal inertial data in body frame (inertia about COM: xx yy zz xy xz yz) */
  float body_mass[LGX_NUM_DYN];
  float body_com[LGX_NUM_DYN][3];
  float body_inertia[LGX_NUM_DYN][6];
  /* contact primitives: sphere (radius > 0) or corner (radius 0) in dyn-body frame */
  int32_t num_points;
  int32_t num_report_bodies;
  int32_t leg_dof;                  /* 3 (4 legs: the arrowhead physics kernel) or 6 (2 legs: the
                                       dense physics kernel); 0 is read as 3 */
  int32_t pad_model;
  float point_pos[LGX_MAX_POINTS][3];
  float point_radius[LGX_MAX_POINTS];
  int32_t point_dyn[LGX_MAX_POINTS];
  int32_t point_report[LGX_MAX_POINTS];
  /* lgx contact / limit model */
  float contact_k, contact_c, friction_c, limit_k, limit_c;
  float ground_friction;            /* terrain static_friction, combined by averaging */
  float gravity[3];
  float sim_dt;                     /* float32(sim.dt) */
} lgx_model;

typedef struct lgx_env_params {
  int32_t num_envs;
  int32_t num_obs;                  /* 48 or 48 + num_height_points */
  int32_t decimation;
  int32_t control_type;             /* enum lgx_control */
  float action_scale, clip_actions, clip_obs;
  float dt;                         /* decimation * sim_dt (legged_robot.py:770) */
  float default_dof_pos[LGX_NUM_DOF];
  float soft_lower[LGX_NUM_DOF], soft_upper[LGX_NUM_DOF];   /* legged_robot.py:306-309 */
  float dof_vel_limits[LGX_NUM_DOF], torque_limits[LGX_NUM_DOF];
  float p_gains[LGX_NUM_DOF], d_gains[LGX_NUM_DOF];
  float soft_dof_vel_limit, soft_torque_limit;
  float max_episode_length;         /* ceil(episode_length_s / dt) = 1001 (legged_robot.py:777) */
  float max_episode_length_s;
  int32_t resample_interval;        /* int(resampling_time / dt) = 500 (legged_robot.py:342) */
  int32_t push_robots;
  int32_t push_interval;            /* ceil(push_interval_s / dt) = 751 (legged_robot.py:779) */
  float max_push_vel_xy;
  int32_t heading_command;
  float cmd_ranges[4][2];           /* lin_vel_x, lin_vel_y, ang_vel_yaw, heading */
  float obs_scale_lin_vel, obs_scale_ang_vel, obs_scale_dof_pos, obs_scale_dof_vel, obs_scale_height;
  int32_t add_noise;
  float noise_scale_vec[LGX_MAX_OBS];   /* _get_noise_scale_vec (legged_robot.py:477-500) */
  /* terrain */
  int32_t terrain_kind;             /* 0 plane/none, 1 heightfield/trimesh (sampled heightfield) */
  int32_t measure_heights;
  int32_t num_height_points;
  float height_points[LGX_MAX_HEIGHT_POINTS][2];  /* base-frame xy (legged_robot.py:802-816) */
  float border_size, horizontal_scale, vertical_scale;
  int32_t curriculum;               /* terrain curriculum (legged_robot.py:443-463) */
  int32_t custom_origins;
  int32_t max_terrain_level;        /* num_rows */
  int32_t terrain_num_cols;
  float terrain_env_length;
  float base_init_state[13];
  /* rewards, in reference evaluation order (alphabetical, non-zero scale, x dt) */
  int32_t num_terms;
  int32_t term_ids[LGX_MAX_TERMS];
  float term_scales[LGX_MAX_TERMS];
  int32_t termination_slot;         /* episode_sums row of "termination" or -1 */
  float termination_scale;
  int32_t only_positive_rewards;
  float tracking_sigma, base_height_target, max_contact_force;
  int32_t num_feet, feet_indices[4];
  int32_t num_penalised, penalised_indices[16];
  int32_t num_termination_bodies, termination_indices[8];
  int32_t send_timeouts;
  /* Go1 actuator-net history (go1.py:50-53,79-107); enabled if use_actuator_history */
  int32_t use_actuator_history;
  float act_pos_err_mean[LGX_NUM_DOF], act_pos_err_std[LGX_NUM_DOF];
  float act_vel_mean[LGX_NUM_DOF], act_vel_std[LGX_NUM_DOF];
  uint64_t seed;
} lgx_env_params;

typedef struct lgx_buffers {
  float* root_states;        /* [N,13] */
  float* dof_state;          /* [N,12,2] */
  float* dof_targets;        /* [N,12] target_poses (legged_robot.py:94) */
  float* torques;            /* [N,12] */
  float* contact_forces;     /* [N,B,3] */
  float* actions;            /* [N,12] clipped actions (input written by host, clipped in place) */
  float* last_actions;       /* [N,12] */
  float* last_dof_vel;       /* [N,12] */
  float* last_root_vel;      /* [N,6] */
  float* commands;           /* [N,4] */
  float* base_lin_vel;       /* [N,3] */
  float* base_ang_vel;       /* [N,3] */
  float* projected_gravity;  /* [N,3] */
  float* feet_air_time;      /* [N,4] */
  float* obs;                /* [N,num_obs] */
  float* rew;                /* [N] */
  uint8_t* reset;            /* [N] bool */
  uint8_t* time_out;         /* [N] bool */
  int64_t* episode_length;   /* [N] */
  float* episode_sums;       /* [T,N]  T = num_terms (+1 if termination) */
  float* measured_heights;   /* [N,P] */
  float* env_origins;        /* [N,3] */
  int64_t* terrain_levels;   /* [N] */
  int64_t* terrain_types;    /* [N] */
  float* terrain_origins;    /* [rows, cols, 3] */
  const int16_t* height_samples; /* [hf_rows, hf_cols] */
  int32_t hf_rows, hf_cols;
  float* body_mass_scale;    /* [N,13] per-env mass / nominal mass (domain randomisation) */
  float* friction;           /* [N] per-env shape friction */
  float* act_hist;           /* [N,12,2,5] actuator-net history (pos_err, vel) oldest..newest */
  float* model_ins;          /* [decimation,N,120] actuator-net inputs per substep */
  const float* act_net_w;    /* packed transposed actuator-MLP weights (lgx_actuator_mlp) or NULL */
  const float* act_net_scale;/* [3] output scale (vel_std per leg joint) */
  float* act_dvel;           /* [decimation,N,12] actuator-net outputs (dVel, go1.py:100-105) */
  float* extras;             /* [T + 2]: episode means per term, terrain_level, reset count */
  uint8_t* extras_time_outs; /* [N] time_outs as last published (stale semantics) */
  float* scratch;            /* [lgx_scratch_floats(N)] reduction partials + completion ticket */
  /* LGX_CTRL_SEA: the packed SEA LSTM (lgx_actuator_lstm layout) and its hidden / cell state
   * [2 layers, N*12 joints, 8] (anymal.py:65-69 sea_hidden_state / sea_cell_state); the state of
   * an env whose episode_length is 0 when a step starts is taken as zero (the reset of
   * anymal.py:56-60: reset envs have episode_length 0 until their next step) */
  const float* sea_w;
  float* sea_h;
  float* sea_c;
  /* trimesh terrain with the slope correction (terrain.py:70-73: convert_heightfield_to_trimesh
   * with slope_treshold): per vertex (i, j) of the heightfield, bits 0-3 = move code
   * (dx + 1) * 3 + (dy + 1) of the corrected mesh (cells, each in {-1, 0, 1}), bit 4 = some vertex
   * of rows i-1 .. i+2, cols j-1 .. j+2 moved (lgx_trimesh_build).  NULL: contact against the
   * sampled heightfield itself (mesh_type heightfield, or no correction). */
  const int8_t* hf_trimesh;
} lgx_buffers;

typedef struct lgx_sim lgx_sim;

const char* lgx_last_error(void);
int lgx_version(void);

/* sizeof(lgx_model), sizeof(lgx_env_params), sizeof(lgx_buffers), sizeof(lgx_mlp_desc),
 * sizeof(lgx_ppo_loss_args), sizeof(lgx_reduce_job), sizeof(lgx_ppo_act_args),
 * sizeof(lgx_ppo_store_args), sizeof(lgx_gemm_args), sizeof(lgx_copy2d_job),
 * sizeof(lgx_gemm_tn_args), sizeof(lgx_mlp_x3_desc): lets bindings verify layout */
void lgx_struct_sizes(int64_t out[12]);

/* Trimesh terrain from the int16 heightfield on the device (isaacgym terrain_utils
 * convert_heightfield_to_trimesh as called at terrain.py:70-73; legged_robot.py:629-643): with
 * height_threshold >= 0 (= slope_treshold * (horizontal_scale / vertical_scale) in height units, the
 * reference's own scaling of cfg.slope_treshold, computed by the caller in double) every vertex
 * whose neighbour along x, y or the cell diagonal is higher by more than it moves one cell toward
 * that neighbour; < 0: no correction.  Writes (each output optional, NULL to skip): vertices
 * float32 [rows * cols, 3] (x = row, y = col on the reference's np.linspace grid in double, + the
 * moves, then rounded to float; z = height * vertical_scale), triangles uint32
 * [2 (rows - 1)(cols - 1), 3] ((v00, v11, v01), (v00, v10, v11) per cell), and the contact table
 * of lgx_buffers.hf_trimesh. */
int lgx_trimesh_build(const int16_t* height_samples, int32_t rows, int32_t cols, double horizontal_scale,
                      double vertical_scale, double height_threshold, float* vertices, uint32_t* triangles,
                      int8_t* contact_table, void* stream);

/* Lanes per leg (1, 2, 4 or 8) of the physics launch at `num_envs` envs, i.e. which
 * lgx_physics_kernel<PP> instantiation lgx_step / lgx_simulate run: 4 at every size (env
 * LGX_PHYS_PP overrides); LGX_EINVAL for num_envs <= 0. */
int32_t lgx_physics_lane_split(int32_t num_envs);

/* Bytes of scratch the caller must bind in lgx_buffers.scratch. */
int64_t lgx_scratch_floats(int32_t num_envs, int32_t num_terms);

/* Replaces gym.create_sim + create_actor loop + prepare_sim + acquire_*_tensor
 * (legged_robot.py:233-249,645-740; base_task.py:85; legged_robot.py:507-524). */
int lgx_sim_create(const lgx_model* model, const lgx_env_params* params, const lgx_buffers* bufs,
                   int device, lgx_sim** out);
int lgx_sim_destroy(lgx_sim* sim);

/* The sim's state tensors by id (SURVEY §8(b) lgx_sim_buffer): the device pointer bound at
 * lgx_sim_create (or the latest lgx_rebind_obs), its shape (ndim <= 4, row-major, contiguous) and
 * element type.  Replaces the gym tensor acquisition + wrap_tensor of the reference
 * (legged_robot.py:507-524: actor_root_state, dof_state, net_contact_force) and the buffers
 * _init_buffers allocates (legged_robot.py:525-565); a binding wraps them without copies (DLPack /
 * from_blob).  Unbound (NULL) buffers are reported with a NULL pointer and their shape. */
enum lgx_buffer_id {
  LGX_BUF_ROOT_STATES = 0,  /* f32 [N,13] */
  LGX_BUF_DOF_STATE,        /* f32 [N,12,2] */
  LGX_BUF_DOF_TARGETS,      /* f32 [N,12] */
  LGX_BUF_TORQUES,          /* f32 [N,12] */
  LGX_BUF_CONTACT_FORCES,   /* f32 [N,LGX_MAX_BODIES,3] */
  LGX_BUF_ACTIONS,          /* f32 [N,12] */
  LGX_BUF_LAST_ACTIONS,     /* f32 [N,12] */
  LGX_BUF_LAST_DOF_VEL,     /* f32 [N,12] */
  LGX_BUF_LAST_ROOT_VEL,    /* f32 [N,6] */
  LGX_BUF_COMMANDS,         /* f32 [N,4] */
  LGX_BUF_BASE_LIN_VEL,     /* f32 [N,3] */
  LGX_BUF_BASE_ANG_VEL,     /* f32 [N,3] */
  LGX_BUF_PROJECTED_GRAVITY,/* f32 [N,3] */
  LGX_BUF_FEET_AIR_TIME,    /* f32 [N,4] */
  LGX_BUF_OBS,              /* f32 [N,num_obs] */
  LGX_BUF_REW,              /* f32 [N] */
  LGX_BUF_RESET,            /* u8 [N] */
  LGX_BUF_TIME_OUT,         /* u8 [N] */
  LGX_BUF_EPISODE_LENGTH,   /* i64 [N] */
  LGX_BUF_EPISODE_SUMS,     /* f32 [T,N], T = num_terms (+1 with a termination slot) */
  LGX_BUF_MEASURED_HEIGHTS, /* f32 [N,num_height_points] */
  LGX_BUF_ENV_ORIGINS,      /* f32 [N,3] */
  LGX_BUF_TERRAIN_LEVELS,   /* i64 [N] */
  LGX_BUF_TERRAIN_TYPES,    /* i64 [N] */
  LGX_BUF_EXTRAS,           /* f32 [T+2] */
  LGX_BUF_COUNT
};
enum lgx_dtype { LGX_F32 = 0, LGX_U8 = 1, LGX_I64 = 2 };
int lgx_sim_buffer(lgx_sim* sim, int32_t buffer_id, void** dev_ptr, int64_t shape[4], int32_t* ndim,
                   int32_t* dtype);

/* Full env step: clip actions, `decimation` x (targets -> physics substep), then the fused
 * post-physics step.  Replaces LeggedRobot.step (legged_robot.py:79-107) including
 * set_dof_position_target_tensor / simulate / refresh_* and post_physics_step.
 * `common_step_counter` is the host counter value AFTER this step's increment. */
int lgx_step(lgx_sim* sim, int64_t common_step_counter, void* stream);

/* lgx_step with the policy's raw actions read from `actions` (device float[N,12], row-major)
 * instead of the bound actions buffer; the clipped actions are still written to the bound
 * buffer (self.actions = clip(actions), legged_robot.py:85-86) -- no host-side copy. */
int lgx_step_from(lgx_sim* sim, const float* actions, int64_t common_step_counter, void* stream);

/* Re-point the observation output (device float[N, num_obs]) for the next calls.  The reference
 * rebinds obs_buf every step (`self.obs_buf = torch.cat(...)`, legged_robot.py:218), so rsl_rl
 * keeps the previous step's tensor alive across env.step(); callers double-buffer with this. */
int lgx_rebind_obs(lgx_sim* sim, float* obs);

/* Data-parallel gradient all-reduce over RCCL (SURVEY §8(b) lgx_allreduce_grads; §8(e): the
 * gradient average of a multi-GPU PPO update, one rank per GPU).  One communicator per rank,
 * created collectively from a unique id that rank 0 draws and the caller distributes (e.g. over
 * its torch.distributed group).  The all-reduce is issued on `stream` itself (in place, float32),
 * so it is ordered by that stream like any kernel.  RCCL is loaded at run time from `rccl_path`
 * (the process's own RCCL, e.g. torch's bundled librccl.so; NULL = librccl.so.1); LGX_EINVAL if it
 * cannot be loaded, LGX_EHIP for an RCCL error (message in lgx_last_error). */
#define LGX_COMM_ID_BYTES 128
enum lgx_reduce_op { LGX_REDUCE_SUM = 0, LGX_REDUCE_AVG = 1 };
typedef struct lgx_comm lgx_comm;
int lgx_comm_unique_id(const char* rccl_path, uint8_t id[LGX_COMM_ID_BYTES]);
int lgx_comm_create(const char* rccl_path, const uint8_t id[LGX_COMM_ID_BYTES], int32_t nranks, int32_t rank,
                    int32_t device, lgx_comm** out);
int lgx_comm_destroy(lgx_comm* comm);
int lgx_allreduce_grads(lgx_comm* comm, float* buf, size_t count, int32_t op, void* stream);

/* Per-call copy of the episode extras (device float[T + 2], lgx_buffers.extras layout) written by
 * the next lgx_step / lgx_post_physics / lgx_reset_idx, stale values included.  The reference
 * publishes fresh tensors in extras["episode"] (legged_robot.py:182-189) that consumers keep
 * (rsl_rl's ep_infos); binding a fresh snapshot per call gives the same semantics without a
 * separate copy.  NULL disables the copy. */
int lgx_rebind_extras(lgx_sim* sim, float* snapshot);

/* The Go1 actuator net of lgx_step runs on an internal stream (its output, actuator dVel, is
 * not consumed by the step: go1.py:71-73) and overlaps post-physics and the caller's next
 * work; the next lgx_step / lgx_simulate orders itself after it.  Make `stream` wait for that
 * work before reading act_dvel on it. */
int lgx_sync_aux(lgx_sim* sim, void* stream);

/* Physics only: `n` substeps with the currently bound dof_targets (gym.simulate x n). */
int lgx_simulate(lgx_sim* sim, int32_t n, void* stream);

/* The drive inputs of lgx_step's physics launch with the dynamics frozen: clip the actions
 * (`actions`, or the bound buffer when NULL) into the bound actions buffer, the position targets
 * (_compute_poses, legged_robot.py:394-397) into dof_targets, `decimation` substeps of the Go1
 * actuator-net history (go1.py:79-98) into act_hist / model_ins, and with LGX_CTRL_SEA
 * `decimation` steps of the SEA LSTM (anymal.py:71-77: sea_h / sea_c advanced, the last substep's
 * torques, clamped to the effort limit, into torques), all from the CURRENT dof state, which stays
 * unchanged (as the reference's decimation loop sees it when the physics does not move: the golden
 * replay).  The actuator-network state (history, LSTM) advances as in that loop; the physical
 * state (root, dof, contacts) does not.  Same device code as the physics launch's load stage. */
int lgx_drive_inputs(lgx_sim* sim, const float* actions, void* stream);

/* The physics launch's ground query for a batch of world points (tests, tools): points [n, 4] =
 * (x, y, z, radius), out [n, 4] = (contact depth, normal xyz) against the bound terrain - the
 * slope-corrected trimesh where lgx_buffers.hf_trimesh flags the cell, else the heightfield
 * triangle under the point; depth <= 0: no contact (its magnitude is then unspecified). */
int lgx_ground_contact(lgx_sim* sim, const float* points, int32_t n, float* out, void* stream);

/* post_physics_step only (legged_robot.py:109-141) on the current state buffers. */
int lgx_post_physics(lgx_sim* sim, int64_t common_step_counter, void* stream);

/* The post-physics half of lgx_step_from exactly as the step issues it after its physics launch
 * (legged_robot.py:100-107 -> post_physics_step :109-141, with Go1's actuator_advance / UniNet,
 * go1.py:79-107): for a task with the Go1 actuator net, ONE launch of post-physics workgroups plus
 * actuator-net workgroups over the step's model_ins rows (into act_dvel); otherwise the same launch
 * as lgx_post_physics.  On the current state buffers, so a golden replay (lgx_drive_inputs, scripted
 * state, this call) pins the product step's own launch to the reference. */
int lgx_post_physics_fused(lgx_sim* sim, int64_t common_step_counter, void* stream);

/* reset_idx for the listed envs (legged_robot.py:150-193): dof/root reset, commands,
 * buffers, episode extras.  env_ids: device int32[n]. */
int lgx_reset_idx(lgx_sim* sim, const int32_t* env_ids, int32_t n, int64_t common_step_counter,
                  int32_t init_done, void* stream);

/* Draw injection for parity tests: device float[N, LGX_DRAW_NOISE + num_obs] or NULL to
 * return to the in-kernel Philox stream. */
int lgx_set_draws(lgx_sim* sim, const float* draws);

/* Go1 actuator MLP (UniNet, go1.py:22-35,100-105): rows of 30 inputs -> 3 outputs,
 * 30-128-128-128-3 tanh MLP on the f32 MFMA (the weight-stationary body the step's post-physics
 * launch runs).  w: packed [W0t b0 W1t b1 W2t b2
 * W3t b3] with W_lt = transposed torch Linear weight ([in x out]).  out = net(in) *
 * out_scale[col] (dVel *= vel_std). */
int lgx_actuator_mlp(const float* in, float* out, int64_t rows, const float* w, const float* out_scale,
                     void* stream);

/* ANYmal SEA LSTM (anymal.py:62-78): 2-layer LSTM(2->8), Linear(8->1), in/out scale;
 * x [M,2], h/c [2,M,8] updated in place, tau [M].  w: packed torch layout. */
int lgx_actuator_lstm(const float* x, float* h, float* c, float* tau, int64_t m, const float* w,
                      void* stream);

/* Fused MLP forward (ActorCritic, rsl_rl; legged_robot_config.py:216-220): y = MLP(x) on
 * f32 MFMA, hidden activation ELU (act=1) or tanh (act=2), last layer linear.
 * dims[0..nl] layer widths (<= 512); weights[l]: transposed [in x out] row-major,
 * biases[l]: [out].  `dims`, `weights`, `biases` are HOST arrays of device pointers. */
int lgx_mlp_forward(const float* x, float* y, int64_t rows, int32_t nl, const int32_t* dims,
                    const float* const* weights, const float* const* biases, int32_t act, void* stream);

/* Batched fused MLP forward: `count` (1 or 2) independent MLPs in ONE launch (rollout: actor
 * mean + critic value).  Same per-network contract as lgx_mlp_forward. */
typedef struct lgx_mlp_desc {
  const float* x;
  float* y;
  int64_t rows;
  int32_t nl;
  int32_t act;
  int32_t dims[7];
  const float* weights[6];
  const float* biases[6];
} lgx_mlp_desc;
int lgx_mlp_forward_batch(const lgx_mlp_desc* descs, int32_t count, void* stream);

/* The same MLP forward (rows-in-LDS fusion of every layer, one or two networks per launch) on
 * split-bf16 MFMA products (f32-accurate, as lgx_gemm_nt's split-bf16 path): the rollout's
 * actor / critic inference (rsl_rl ActorCritic.act / evaluate).  weights[l] = lgx_mlp_x3_split
 * image of layer l's nn.Linear weight [dims[l+1]][dims[l]] (lgx_mlp_x3_weight_elems bf16,
 * 16-byte aligned); dims <= 512; the activations of 32 rows must fit the LDS
 * (lgx_mlp_x3_lds_bytes >= 0). */
typedef struct lgx_mlp_x3_desc {
  const float* x;
  float* y;
  int64_t rows;
  int32_t nl;
  int32_t act;                  /* 1 ELU, 2 tanh (hidden layers; the last layer is linear) */
  int32_t dims[7];
  const uint16_t* weights[6];
  const float* biases[6];
} lgx_mlp_x3_desc;
int64_t lgx_mlp_x3_weight_elems(int32_t n_out, int32_t k_in);
int lgx_mlp_x3_split(const float* W, int32_t n_out, int32_t k_in, uint16_t* dst, void* stream);
/* lgx_mlp_x3_split of every layer of one network in one launch (the rsl_rl ActorCritic MLP's
 * weights after an optimizer step): W[l] is layer l's [dims[l+1], dims[l]] weight, dst[l] its image
 * (lgx_mlp_x3_weight_elems(dims[l+1], dims[l]) bf16), nl <= 6. */
int lgx_mlp_x3_split_layers(const float* const* W, const int32_t* dims, int32_t nl, uint16_t* const* dst,
                            void* stream);
int64_t lgx_mlp_x3_lds_bytes(const lgx_mlp_x3_desc* descs, int32_t count);   /* -1: unsupported */
int lgx_mlp_x3_forward(const lgx_mlp_x3_desc* descs, int32_t count, void* stream);

/* In-library kernel timing for the measurement harness (bench.py): with `period` = k > 0, every
 * k-th lgx_step dispatches its kernels through hipExtLaunchKernelGGL with a (start, stop)
 * hipEvent pair per kernel class (0 physics, 1 actuator MLP, 2 post-physics kernel); 0 turns
 * timing off.  lgx_profile_collect synchronises those events (call it OUTSIDE timed regions),
 * writes per class the summed milliseconds and launch count to ms[3] / count[3], and clears
 * the record. */
int lgx_profile_enable(lgx_sim* sim, int32_t period);
int lgx_profile_collect(lgx_sim* sim, double* ms, int64_t* count);

/* Cross-stream ordering events of the PPO update (the dW GEMMs on a second stream next to the dA
 * GEMMs): hipEventDisableTiming | hipEventDisableSystemFence - the release / acquire stay at device
 * scope (every consumer is a kernel on the same GPU; an RCCL send is a kernel on it too), so a
 * record does not write back and invalidate the caches to system scope the way a default event
 * does.  The PPO update uses them in single-process runs; data-parallel runs keep system-scope
 * events (their joins also order buffers that RCCL peers write).  `*ev` receives a hipEvent_t. */
int lgx_event_create(void** ev);
int lgx_event_destroy(void* ev);
int lgx_event_record(void* ev, void* stream);
int lgx_stream_wait_event(void* stream, void* ev);
/* Record `ev` with the completion of the next lgx kernel launch of the calling thread (bound to the
 * dispatch: no separate record packet on the producer stream); lgx_launch_bind_pending returns 1
 * when no launch has taken it yet (record it with lgx_event_record then) and disarms. */
int lgx_launch_bind_event(void* ev);
int lgx_launch_bind_pending(void);

/* Generalised advantage estimation (rsl_rl RolloutStorage.compute_returns, before the
 * advantage normalisation): rewards/values/dones [T,N] (dones uint8), last_values [N] ->
 * returns, advantages (= returns - values) [T,N]. */
int lgx_gae(const float* rewards, const float* values, const uint8_t* dones, const float* last_values, float* returns,
            float* advantages, int32_t T, int32_t N, float gamma, float lam, void* stream);

/* lgx_gae followed by the advantage normalisation of rsl_rl v1.0.x RolloutStorage.compute_returns
 * (external to the reference; called from on_policy_runner.learn, which scripts/train.py:43 runs):
 * `(adv - adv.mean()) / (adv.std() + 1e-8)`, unbiased std, in place (single process) - two
 * launches instead of the GAE kernel + the torch mean / std / elementwise chain.  scratch:
 * lgx_gae_norm_scratch(N) doubles of device memory (per-workgroup count / mean / M2, combined in a
 * fixed order with Chan's pairwise formula: no cancellation when |mean| >> std). */
int64_t lgx_gae_norm_scratch(int32_t N);
int lgx_gae_norm(const float* rewards, const float* values, const uint8_t* dones, const float* last_values,
                 float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam, double* scratch,
                 void* stream);

/* The data-parallel form of lgx_gae_norm (global statistics over every rank's advantages, as one
 * process holding all ranks' envs would normalise): lgx_gae_parts runs the GAE and writes this
 * rank's per-workgroup (count, mean, M2) summaries, lgx_gae_norm_scratch(N) doubles, to `parts`;
 * the host gathers every rank's parts (torch.distributed all_gather, rank order) and
 * lgx_adv_norm normalises this rank's n = T*N advantages in place with the statistics of the
 * `nparts` gathered summaries (combined in order, so every rank applies the same mean / std; at
 * world 1 the result is bitwise lgx_gae_norm's). */
int lgx_gae_parts(const float* rewards, const float* values, const uint8_t* dones, const float* last_values,
                  float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam, double* parts,
                  void* stream);
int lgx_adv_norm(float* advantages, int64_t n, const double* parts, int32_t nparts, void* stream);

/* ---- PPO update (rsl_rl PPO.update, legged_robot_config.py:226-239): the non-GEMM work of a
 * minibatch step.  Activations are net-major [2 (actor, critic), M, H]; the GEMMs between
 * these calls are library GEMMs issued by the host.  All pointers are device pointers. */
#define LGX_PPO_MAX_ACTIONS 16
#define LGX_MAX_REDUCE_JOBS 16

/* PPO.act + RolloutStorage.add_transitions of one env step: actions = mu + std * noise,
 * log-prob, storage row (st_* point at row t of the [T, N, .] storage tensors). */
typedef struct lgx_ppo_act_args {
  int64_t num_envs;
  int32_t num_actions, num_obs, num_cobs, pad;
  const float* mu;              /* [N,A] actor mean (rollout MLP output) */
  const float* value;           /* [N]   critic value, or NULL when the critic wrote st_values itself */
  const float* std;             /* [A] */
  const float* noise;           /* [N,A] standard-normal draws */
  const float* obs;             /* [N,num_obs] */
  const float* cobs;            /* [N,num_cobs] privileged obs or NULL */
  float* actions_out;           /* [N,A] */
  float* st_obs;
  float* st_cobs;               /* NULL iff cobs is NULL */
  float* st_actions;
  float* st_values;
  float* st_logp;
  float* st_mu;
  float* st_sigma;
} lgx_ppo_act_args;
int lgx_ppo_act(const lgx_ppo_act_args* args, void* stream);

/* PPO.process_env_step: st_rew = rew + gamma * st_values * time_outs; st_dones = reset */
typedef struct lgx_ppo_store_args {
  int64_t num_envs;
  float gamma;
  int32_t pad;
  const float* rew;
  const uint8_t* reset;
  const uint8_t* time_outs;     /* NULL: no time-out bootstrap */
  const float* st_values;
  float* st_rew;
  uint8_t* st_dones;
} lgx_ppo_store_args;
int lgx_ppo_store(const lgx_ppo_store_args* args, void* stream);
/* lgx_ppo_act of step t+1 and the deferred lgx_ppo_store of step t in ONE launch (rsl_rl
 * PPO.act + PPO.process_env_step of the runner's collection loop; the store reads only step t's
 * env outputs and storage row t, which the act does not touch); same envs. */
int lgx_ppo_act_store(const lgx_ppo_act_args* args, const lgx_ppo_store_args* prev, void* stream);
/* The rollout step's policy inference and lgx_ppo_act_store in ONE launch (rsl_rl PPO.act:
 * ActorCritic.act + evaluate + RolloutStorage.add_transitions, and process_env_step of the previous
 * step): lgx_mlp_x3_forward of descs[0] (actor, output = the action means into descs[0].y) and
 * descs[1] (critic, output = the storage values row) with lgx_ppo_act's arithmetic done in the
 * actor's last-layer epilogue; bit-identical rows to lgx_mlp_x3_forward + lgx_ppo_act(_store).
 * count == 2, rows == args->num_envs, num_actions <= LGX_PPO_MAX_ACTIONS, args->value NULL, args->mu
 * unused (the means come from the epilogue); prev NULL: no store. */
int lgx_mlp_x3_forward_act(const lgx_mlp_x3_desc* descs, int32_t count, const lgx_ppo_act_args* args,
                           const lgx_ppo_store_args* prev, void* stream);

/* dst[r, :] = src[idx[r], :] for r < rows (minibatch gather of storage rows) */
int lgx_ppo_gather_rows(const float* src, float* dst, const int64_t* idx, int64_t rows, int32_t width, void* stream);

/* z[n, r, c] = act(z[n, r, c] + b[n, c]) in place; act 0 none, 1 ELU, 2 tanh; cols % 4 == 0 */
int lgx_bias_act(float* z, const float* b, int64_t rows, int32_t cols, int32_t nets, int32_t act, void* stream);

typedef struct lgx_ppo_loss_args {
  int64_t rows;                 /* M, minibatch size */
  int32_t num_actions;          /* A <= LGX_PPO_MAX_ACTIONS */
  int32_t use_clipped_value_loss;
  float clip_param, value_loss_coef, entropy_coef;
  const int64_t* idx;           /* storage row of minibatch row r (NULL: identity) */
  const float* mu_raw;          /* [M,A] actor output before its bias (head_in == NULL) */
  const float* v_raw;           /* [M]   critic output before its bias (head_in == NULL) */
  const float* b4a;             /* [A] */
  const float* b4c;             /* [1] */
  const float* std;             /* [A] action std parameter */
  /* storage (indexed by idx): */
  const float* actions;         /* [*,A] */
  const float* old_logp;        /* [*] */
  const float* old_mu;          /* [*,A] */
  const float* old_sigma;       /* [*,A] */
  const float* advantages;      /* [*] normalised */
  const float* target_values;   /* [*] */
  const float* returns;         /* [*] */
  /* outputs */
  float* d_mu;                  /* [M,A] d loss / d mu */
  float* d_v;                   /* [M]   d loss / d value */
  float* partials;              /* [lgx_ppo_loss_partials_floats(M, A)] */
  float* g_std;                 /* [A] gradient slots in the flat gradient buffer */
  float* g_b4a;                 /* [A] */
  float* g_b4c;                 /* [1] */
  float* stats;                 /* [3]: KL mean (this minibatch), += surrogate mean, += value-loss mean */
  /* non-NULL: rsl_rl's adaptive schedule applied on the device from this minibatch's KL in the
   * same call (lgx_ppo_adapt_lr semantics, kl_scale 1); NULL: the caller adapts separately
   * (data-parallel: after the all-reduce of the KL) */
  double* lr;
  double desired_kl;
  /* non-NULL: the output layers are evaluated in the same call (mu_raw, v_raw unused):
   * head_in = last hidden activations [2, M, hidden] (actor, critic), W4a [A, hidden],
   * W4c [1, hidden]; hidden % 16 == 0, (A + 1) * hidden * 4 <= 64 KB */
  const float* head_in;
  const float* W4a;
  const float* W4c;
  int32_t hidden;
  /* nonzero: lgx_ppo_loss leaves the partial reduction (gradient slots, stats, adaptive LR) to
   * the following lgx_head_bwd_finalize call, which runs it on one extra workgroup */
  int32_t defer_finalize;
} lgx_ppo_loss_args;
int64_t lgx_ppo_loss_partials_floats(int64_t rows, int32_t num_actions);
/* loss = mean(max(-adv r, -adv clip(r))) + c_v mean(value loss) - c_e mean(entropy), with its
 * gradient (torch autograd tie conventions) and the adaptive-schedule KL */
int lgx_ppo_loss(const lgx_ppo_loss_args* args, void* stream);

/* adaptive schedule on the device: lr (double) from KL = kl_sum[0] * kl_scale */
int lgx_ppo_adapt_lr(const float* kl_sum, float kl_scale, double* lr, double desired_kl, void* stream);

/* output layers backward: partials per 32-row chunk [A*H dW4a | H dW4c | 2H db3] (H <= 1024);
 * A3 [2,M,H] (post-ELU) is overwritten by dZ3 */
int64_t lgx_head_bwd_partials_floats(int64_t rows, int32_t num_actions, int32_t hidden);
int lgx_head_bwd(const float* d_mu, const float* d_v, const float* W4a, const float* W4c, float* A3, int64_t rows,
                 int32_t num_actions, int32_t hidden, float* partials, void* stream);
/* lgx_head_bwd plus the finalize of a deferred lgx_ppo_loss call (loss->defer_finalize != 0,
 * same rows / actions) on one extra workgroup of the same launch */
int lgx_head_bwd_finalize(const lgx_ppo_loss_args* loss, const float* d_mu, const float* d_v, const float* W4a,
                          const float* W4c, float* A3, int64_t rows, int32_t num_actions, int32_t hidden,
                          float* partials, void* stream);

/* lgx_ppo_loss (head_in form) and lgx_head_bwd in ONE launch over 32-row chunks: the last hidden
 * activations are read once; head_in ([2,M,hidden], hidden % 16 == 0) is overwritten by dZ3;
 * args->partials takes out[0] floats of loss partials, head_partials out[1] floats of
 * [A*H dW4a | H dW4c | 2H db3] chunk partials (lgx_ppo_loss_bwd_layout; out[2] = dynamic LDS
 * bytes, <= 96 KB).  d_mu / d_v are not written.  With args->defer_finalize the loss finalize
 * runs in the following lgx_reduce_slices_finalize call.  Replaces lgx_ppo_loss +
 * lgx_head_bwd_finalize (rsl_rl ppo.py:154-185 + the output layers' backward). */
int lgx_ppo_loss_bwd_layout(int64_t rows, int32_t num_actions, int32_t hidden, int64_t out[3]);
int lgx_ppo_loss_bwd(const lgx_ppo_loss_args* args, float* head_partials, void* stream);

/* dA [nets,M,H] -> dA * elu'(Y) in place (Y = ELU output) + per-chunk column sums */
int64_t lgx_colsum_partials_floats(int64_t rows, int32_t hidden, int32_t nets);
int lgx_elu_bwd_colsum(float* dA, const float* Y, int64_t rows, int32_t hidden, int32_t nets, float* partials,
                       void* stream);

/* dst[j*dst_stride + i] = sum_{s<slices} src[j*job_stride + s*slice_stride + i], i < n, j < count */
typedef struct lgx_reduce_job {
  const float* src;
  float* dst;
  int64_t n, job_stride, slice_stride, dst_stride;
  int32_t slices, count;
} lgx_reduce_job;
int lgx_reduce_slices(const lgx_reduce_job* jobs, int32_t njobs, void* stream);
/* lgx_reduce_slices plus the deferred loss finalize of a lgx_ppo_loss_bwd call (one extra
 * workgroup; loss->defer_finalize != 0): d std, head-bias gradients, KL, stats, adaptive LR */
int lgx_reduce_slices_finalize(const lgx_reduce_job* jobs, int32_t njobs, const lgx_ppo_loss_args* loss,
                               void* stream);
/* lgx_reduce_slices (loss == NULL) / lgx_reduce_slices_finalize (loss != NULL) that also writes
 * sq[w] = the sum of squares of the gradient values workgroup w writes (the finalize workgroup:
 * d std and the head-bias gradients; fixed summation order), w < lgx_reduce_slices_blocks(jobs,
 * njobs, loss != NULL); with step != NULL (needs loss) the finalize workgroup also advances the
 * optimizer step.  The clip norm of torch's clip_grad_norm_ then needs no pass of its own over the
 * gradient (lgx_adam_clip_mirror_sq); single-process updates (a data-parallel gradient is
 * all-reduced after its reduction) */
int64_t lgx_reduce_slices_blocks(const lgx_reduce_job* jobs, int32_t njobs, int32_t with_finalize);
int lgx_reduce_slices_sq(const lgx_reduce_job* jobs, int32_t njobs, const lgx_ppo_loss_args* loss, float* sq,
                         int64_t* step, void* stream);

/* clip_grad_norm_(max_norm) of (grad_scale * g) fused into torch-Adam (no weight decay) over
 * one flat parameter buffer; *step is advanced on the device; lr is a device double */
int lgx_adam_clip(float* p, float* g, float* m, float* v, int64_t n, float* partials, int32_t nparts, float grad_scale,
                  float max_norm, const double* lr, int64_t* step, float beta1, float beta2, float eps, void* stream);

/* ---- Fused f32-MFMA GEMMs of the PPO update (lgx_gemm.hip, hand-written for gfx950).
 * Replace the library GEMM + lgx_bias_act (forward) and GEMM + lgx_elu_bwd_colsum (backward)
 * pairs of a minibatch step (rsl_rl PPO.update, legged_robot_config.py:226-239):
 *   C[z][m][n] = epi( sum_k A[z*sa + m*lda + k] * B[z*sb + n*ldb + k] ),  z < batch
 *   LGX_GEMM_PLAIN        epi(x) = x
 *   LGX_GEMM_BIAS_ELU     epi(x) = ELU(x + bias[z*N + n])
 *   LGX_GEMM_DELU_COLSUM  C = x * ELU'(Y) with Y (same layout as C) the ELU output, and
 *                         partials[t][z*N + n] = sum of C over rows 128t .. 128t+127
 *   LGX_GEMM_DELU         C = x * ELU'(Y) (no column sums: lgx_gemm_tn's colsum of the next
 *                         weight-gradient product gives them); split-bf16 with a pre-split B and
 *                         K % 32 == 0 only
 * Requirements: N % 128 == 0, K % 4 == 0, A/B 16-byte aligned with lda, ldb, sa, sb % 4 == 0
 * (pad K with zero columns).  sa may be 0 (one input shared by the batch). */
/* algo: LGX_GEMM_ALGO_DEFAULT = the process default (env LGX_GEMM_ALGO = "split" | "f32",
 * "split" when unset); LGX_GEMM_ALGO_F32 = v_mfma_f32_32x32x2_f32 (exact f32 fmaf chain);
 * LGX_GEMM_ALGO_SPLIT_BF16 = each f32 operand split into three RNE bf16 limbs, the six limb
 * products of order <= 2 on v_mfma_f32_32x32x16_bf16 with f32 accumulation (f32-accurate:
 * dropped terms and split residues <= ~2^-25 |a b|, below one f32 product rounding) */
#define LGX_GEMM_ALGO_DEFAULT 0
#define LGX_GEMM_ALGO_F32 1
#define LGX_GEMM_ALGO_SPLIT_BF16 2
#define LGX_GEMM_PLAIN 0
#define LGX_GEMM_BIAS_ELU 1
#define LGX_GEMM_DELU_COLSUM 2
#define LGX_GEMM_DELU 3
typedef struct lgx_gemm_args {
  int64_t M;
  int32_t N, K, batch, epi;
  const float* A;
  int64_t lda, sa;
  const float* B;
  int64_t ldb, sb;
  float* C;
  int64_t ldc, sc;
  const float* bias;            /* [batch][N] (BIAS_ELU) */
  const float* Y;               /* like C (DELU_COLSUM) */
  float* partials;              /* [lgx_gemm_partials_floats(M, N, batch)] (DELU_COLSUM) */
  int32_t algo;                 /* LGX_GEMM_ALGO_*: how the f32 products are evaluated */
  int32_t tile_rows;            /* pipelined split-bf16 kernel: 0 = automatic, 128 / 256 forces the
                                   output tile height */
  const uint16_t* Bs;           /* split-bf16 only, optional: B pre-split by lgx_split_bf16 into
                                   [batch][N][ceil(K/32)][3 limbs][32] bf16 (then B is not read) */
} lgx_gemm_args;
int64_t lgx_gemm_partials_floats(int64_t M, int32_t N, int32_t batch);
int lgx_gemm_nt(const lgx_gemm_args* args, void* stream);


/* Weight-gradient GEMM of the PPO update (the dW_k = dZ_k^T Y_{k-1} products of rsl_rl's
 * backward, legged_robot_config.py:226-239), split-K over row slices, split-bf16 products
 * (f32-accurate, as LGX_GEMM_ALGO_SPLIT_BF16):
 *   C[((z * slices + s) * R + n) * ldc + c] = sum_{m = s Ms}^{(s+1) Ms - 1} A[z*sa + m*lda + n] * B[z*sb + m*ldb + c]
 * for z < batch, s < slices, n < R, c < Cc, Ms = M / slices.  Requirements: Ms % 32 == 0,
 * R % 128 == 0, ldb >= Cc rounded up to 128 (the padding columns are read, not stored), A/B
 * 16-byte aligned with lda, ldb, sa, sb % 4 == 0.  lgx_reduce_slices then sums the slices.
 * colsum (optional, NULL to skip): colsum[(z * slices + s) * R + n] = sum over the same rows of
 * A[z*sa + m*lda + n] - the per-slice column sums of A, i.e. with A = dZ_k the bias gradient's
 * partials (rsl_rl's db_k), computed from the f32 rows the kernel stages anyway. */
typedef struct lgx_gemm_tn_args {
  int64_t M;                    /* rows per batch entry */
  int32_t R, Cc, slices, batch;
  const float* A;
  int64_t lda, sa;
  const float* B;
  int64_t ldb, sb;
  float* C;
  int64_t ldc;
  float* colsum;                /* [batch][slices][R] or NULL */
} lgx_gemm_tn_args;
int lgx_gemm_tn(const lgx_gemm_tn_args* args, void* stream);

/* weight preparation for lgx_gemm_nt: dst[b][r][c] = src[b][r][c] (transpose 0) or
 * dst[b][c][r] = src[b][r][c] (transpose 1), r < rows, c < cols; dst padding is untouched */
typedef struct lgx_copy2d_job {
  const float* src;
  float* dst;
  int64_t src_ld, src_bs, dst_ld, dst_bs;
  int32_t rows, cols, batch, transpose;
} lgx_copy2d_job;
int lgx_copy2d(const lgx_copy2d_job* jobs, int32_t njobs, void* stream);

/* GEMM operand pre-split for the split-bf16 path: per job (lgx_copy2d_job), the logical operand
 * out[b][n][k] = transpose ? src[b][k][n] : src[b][n][k] (bit 0 of `transpose`) written as RNE
 * bf16 limbs x0 + x1 + x2 at dst[b*dst_bs + n*dst_ld + (k/32)*96 + limb*32 + k%32] (uint16
 * units; dst_ld >= lgx_split_bf16_elems(1, K)), zero-filled for K <= k < ceil(K/32)*32 */
int64_t lgx_split_bf16_elems(int32_t n, int32_t k);
int lgx_split_bf16(const lgx_copy2d_job* jobs, int32_t njobs, void* stream);

/* lgx_adam_clip that also writes every updated parameter of the `mirrors` blocks (lgx_copy2d
 * job layout; src = a contiguous block of p) into its derived copy (zero-padded / transposed
 * GEMM operands), replacing the lgx_copy2d pass before the next minibatch; <= LGX_MAX_REDUCE_JOBS mirrors.
 * A mirror with bit 1 of `transpose` set writes the lgx_split_bf16 limb layout instead (bit 0:
 * transposed), keeping pre-split split-bf16 GEMM operands current */
int lgx_adam_clip_mirror(float* p, float* g, float* m, float* v, int64_t n, float* partials, int32_t nparts,
                         float grad_scale, float max_norm, const double* lr, int64_t* step, float beta1, float beta2,
                         float eps, const lgx_copy2d_job* mirrors, int32_t nmirrors, void* stream);
/* lgx_adam_clip_mirror on the nsq sums of squares written by lgx_reduce_slices_sq calls (the step
 * advanced there too): no sum-of-squares launch; grad_scale 1 */
int lgx_adam_clip_mirror_sq(float* p, float* g, float* m, float* v, int64_t n, const float* sq, int32_t nsq,
                            float max_norm, const double* lr, int64_t* step, float beta1, float beta2, float eps,
                            const lgx_copy2d_job* mirrors, int32_t nmirrors, void* stream);

/* lgx_ppo_gather_rows into rows of dst_ld floats, columns width .. dst_ld-1 zero-filled */
int lgx_ppo_gather_rows_padded(const float* src, float* dst, const int64_t* idx, int64_t rows, int32_t width,
                               int32_t dst_ld, void* stream);
/* lgx_ppo_gather_rows_padded with every block of `block` rows written twice, back to back
 * (dst = [rows / block][2][block][dst_ld]): per minibatch one [2, M, dst_ld] operand for the
 * batched actor + critic layer-1 weight-gradient GEMM over the same input rows */
int lgx_ppo_gather_rows_padded_dup(const float* src, float* dst, const int64_t* idx, int64_t rows, int32_t width,
                                   int32_t dst_ld, int64_t block, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LGX_H */
