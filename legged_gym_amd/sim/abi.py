"""ctypes mirror of include/lgx.h (the C-ABI of liblgx.so).

The struct layouts below must match the header field for field; `check_layout(lib)` compares
them with the library's own `lgx_struct_sizes` so a drift fails loudly at load time.
This module only describes the ABI; loading the product library is `legged_gym_amd.sim.lib`.
"""
import ctypes as C

NUM_DOF = 12
NUM_DYN = 13
MAX_BODIES = 17
MAX_POINTS = 128
MAX_OBS = 256
MAX_HEIGHT_POINTS = 192
MAX_TERMS = 24
ENV_BLOCK = 4    # smallest envs-per-workgroup the post-physics kernel is built with (sizes scratch)

# reward term ids (enum lgx_reward_term) keyed by the reference's `_reward_<name>` suffix
REWARD_IDS = {
    "lin_vel_z": 0, "ang_vel_xy": 1, "orientation": 2, "base_height": 3, "torques": 4, "energy": 5,
    "dof_vel": 6, "dof_acc": 7, "action_rate": 8, "collision": 9, "termination": 10,
    "dof_pos_limits": 11, "dof_vel_limits": 12, "torque_limits": 13, "tracking_lin_vel": 14,
    "tracking_ang_vel": 15, "feet_air_time": 16, "stumble": 17, "stand_still": 18,
    "feet_contact_forces": 19, "hip_motion": 20, "no_fly": 21,
}
CTRL = {"POS_DRIVE": 0, "P": 1, "V": 2, "T": 3, "SEA": 4}

DRAW_CMD, DRAW_PUSH, DRAW_RESET_DOF, DRAW_RESET_XY = 0, 3, 5, 17
DRAW_RESET_VEL, DRAW_RESET_CMD, DRAW_CURRIC, DRAW_NOISE = 19, 25, 28, 32

f32, i32, i64, u64 = C.c_float, C.c_int32, C.c_int64, C.c_uint64
PF, PU8, PI64, PI16, PI32 = C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(C.c_int64), C.POINTER(C.c_int16), C.POINTER(C.c_int32)


class LgxModel(C.Structure):
    _fields_ = [
        ("joint_rot", f32 * 9 * NUM_DOF), ("joint_pos", f32 * 3 * NUM_DOF), ("joint_axis", f32 * 3 * NUM_DOF),
        ("dof_lower", f32 * NUM_DOF), ("dof_upper", f32 * NUM_DOF), ("dof_vel_limit", f32 * NUM_DOF),
        ("dof_effort", f32 * NUM_DOF), ("kp", f32 * NUM_DOF), ("kd", f32 * NUM_DOF),
        ("body_mass", f32 * NUM_DYN), ("body_com", f32 * 3 * NUM_DYN), ("body_inertia", f32 * 6 * NUM_DYN),
        ("num_points", i32), ("num_report_bodies", i32), ("leg_dof", i32), ("pad_model", i32),
        ("point_pos", f32 * 3 * MAX_POINTS), ("point_radius", f32 * MAX_POINTS),
        ("point_dyn", i32 * MAX_POINTS), ("point_report", i32 * MAX_POINTS),
        ("contact_k", f32), ("contact_c", f32), ("friction_c", f32), ("limit_k", f32), ("limit_c", f32),
        ("ground_friction", f32), ("gravity", f32 * 3), ("sim_dt", f32),
    ]


class LgxEnvParams(C.Structure):
    _fields_ = [
        ("num_envs", i32), ("num_obs", i32), ("decimation", i32), ("control_type", i32),
        ("action_scale", f32), ("clip_actions", f32), ("clip_obs", f32), ("dt", f32),
        ("default_dof_pos", f32 * NUM_DOF), ("soft_lower", f32 * NUM_DOF), ("soft_upper", f32 * NUM_DOF),
        ("dof_vel_limits", f32 * NUM_DOF), ("torque_limits", f32 * NUM_DOF),
        ("p_gains", f32 * NUM_DOF), ("d_gains", f32 * NUM_DOF),
        ("soft_dof_vel_limit", f32), ("soft_torque_limit", f32),
        ("max_episode_length", f32), ("max_episode_length_s", f32),
        ("resample_interval", i32), ("push_robots", i32), ("push_interval", i32), ("max_push_vel_xy", f32),
        ("heading_command", i32), ("cmd_ranges", f32 * 2 * 4),
        ("obs_scale_lin_vel", f32), ("obs_scale_ang_vel", f32), ("obs_scale_dof_pos", f32),
        ("obs_scale_dof_vel", f32), ("obs_scale_height", f32),
        ("add_noise", i32), ("noise_scale_vec", f32 * MAX_OBS),
        ("terrain_kind", i32), ("measure_heights", i32), ("num_height_points", i32),
        ("height_points", f32 * 2 * MAX_HEIGHT_POINTS),
        ("border_size", f32), ("horizontal_scale", f32), ("vertical_scale", f32),
        ("curriculum", i32), ("custom_origins", i32), ("max_terrain_level", i32), ("terrain_num_cols", i32),
        ("terrain_env_length", f32), ("base_init_state", f32 * 13),
        ("num_terms", i32), ("term_ids", i32 * MAX_TERMS), ("term_scales", f32 * MAX_TERMS),
        ("termination_slot", i32), ("termination_scale", f32), ("only_positive_rewards", i32),
        ("tracking_sigma", f32), ("base_height_target", f32), ("max_contact_force", f32),
        ("num_feet", i32), ("feet_indices", i32 * 4),
        ("num_penalised", i32), ("penalised_indices", i32 * 16),
        ("num_termination_bodies", i32), ("termination_indices", i32 * 8),
        ("send_timeouts", i32), ("use_actuator_history", i32),
        ("act_pos_err_mean", f32 * NUM_DOF), ("act_pos_err_std", f32 * NUM_DOF),
        ("act_vel_mean", f32 * NUM_DOF), ("act_vel_std", f32 * NUM_DOF),
        ("seed", u64),
    ]


BUFFER_FIELDS = [
    ("root_states", PF), ("dof_state", PF), ("dof_targets", PF), ("torques", PF), ("contact_forces", PF),
    ("actions", PF), ("last_actions", PF), ("last_dof_vel", PF), ("last_root_vel", PF), ("commands", PF),
    ("base_lin_vel", PF), ("base_ang_vel", PF), ("projected_gravity", PF), ("feet_air_time", PF),
    ("obs", PF), ("rew", PF), ("reset", PU8), ("time_out", PU8), ("episode_length", PI64),
    ("episode_sums", PF), ("measured_heights", PF), ("env_origins", PF), ("terrain_levels", PI64),
    ("terrain_types", PI64), ("terrain_origins", PF), ("height_samples", PI16), ("hf_rows", i32), ("hf_cols", i32),
    ("body_mass_scale", PF), ("friction", PF), ("act_hist", PF), ("model_ins", PF),
    ("act_net_w", PF), ("act_net_scale", PF), ("act_dvel", PF),
    ("extras", PF), ("extras_time_outs", PU8), ("scratch", PF),
    ("sea_w", PF), ("sea_h", PF), ("sea_c", PF), ("hf_trimesh", C.POINTER(C.c_int8)),
]


class LgxBuffers(C.Structure):
    _fields_ = BUFFER_FIELDS


class LgxMlpDesc(C.Structure):
    _fields_ = [("x", C.c_void_p), ("y", C.c_void_p), ("rows", i64), ("nl", i32), ("act", i32), ("dims", i32 * 7),
                ("weights", C.c_void_p * 6), ("biases", C.c_void_p * 6)]


class LgxMlpX3Desc(C.Structure):
    _fields_ = [("x", C.c_void_p), ("y", C.c_void_p), ("rows", i64), ("nl", i32), ("act", i32), ("dims", i32 * 7),
                ("weights", C.c_void_p * 6), ("biases", C.c_void_p * 6)]


class LgxPpoLossArgs(C.Structure):
    _fields_ = [("rows", i64), ("num_actions", i32), ("use_clipped_value_loss", i32), ("clip_param", C.c_float),
                ("value_loss_coef", C.c_float), ("entropy_coef", C.c_float)] + [
        (n, C.c_void_p) for n in ("idx", "mu_raw", "v_raw", "b4a", "b4c", "std", "actions", "old_logp", "old_mu",
                                  "old_sigma", "advantages", "target_values", "returns", "d_mu", "d_v", "partials",
                                  "g_std", "g_b4a", "g_b4c", "stats", "lr")] + [("desired_kl", C.c_double)] + [
        (n, C.c_void_p) for n in ("head_in", "W4a", "W4c")] + [("hidden", i32), ("defer_finalize", i32)]


class LgxReduceJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("n", i64), ("job_stride", i64), ("slice_stride", i64),
                ("dst_stride", i64), ("slices", i32), ("count", i32)]


class LgxPpoActArgs(C.Structure):
    _fields_ = [("num_envs", i64), ("num_actions", i32), ("num_obs", i32), ("num_cobs", i32), ("pad", i32)] + [
        (n, C.c_void_p) for n in ("mu", "value", "std", "noise", "obs", "cobs", "actions_out", "st_obs", "st_cobs",
                                  "st_actions", "st_values", "st_logp", "st_mu", "st_sigma")]


class LgxPpoStoreArgs(C.Structure):
    _fields_ = [("num_envs", i64), ("gamma", C.c_float), ("pad", i32)] + [
        (n, C.c_void_p) for n in ("rew", "reset", "time_outs", "st_values", "st_rew", "st_dones")]


class LgxGemmArgs(C.Structure):
    _fields_ = [("M", i64), ("N", i32), ("K", i32), ("batch", i32), ("epi", i32),
                ("A", C.c_void_p), ("lda", i64), ("sa", i64), ("B", C.c_void_p), ("ldb", i64), ("sb", i64),
                ("C", C.c_void_p), ("ldc", i64), ("sc", i64), ("bias", C.c_void_p), ("Y", C.c_void_p),
                ("partials", C.c_void_p), ("algo", i32), ("tile_rows", i32), ("Bs", C.c_void_p)]


class LgxGemmTnArgs(C.Structure):
    _fields_ = [("M", i64), ("R", i32), ("Cc", i32), ("slices", i32), ("batch", i32),
                ("A", C.c_void_p), ("lda", i64), ("sa", i64), ("B", C.c_void_p), ("ldb", i64), ("sb", i64),
                ("C", C.c_void_p), ("ldc", i64), ("colsum", C.c_void_p)]


class LgxCopy2dJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("src_ld", i64), ("src_bs", i64), ("dst_ld", i64),
                ("dst_bs", i64), ("rows", i32), ("cols", i32), ("batch", i32), ("transpose", i32)]


PPO_MAX_ACTIONS = 16
MAX_REDUCE_JOBS = 16
GEMM_PLAIN, GEMM_BIAS_ELU, GEMM_DELU_COLSUM, GEMM_DELU = 0, 1, 2, 3
GEMM_ALGO_DEFAULT, GEMM_ALGO_F32, GEMM_ALGO_SPLIT_BF16 = 0, 1, 2
GEMM_TILE_M, GEMM_TILE_N, GEMM_K_STEP = 128, 128, 32   # K step: layer-1 rows padded to 1024 B (aligned 128-B lines)


def declare(lib, prefix="lgx"):
    """Attach argtypes/restypes of the product C-ABI to a loaded CDLL."""
    vp = C.c_void_p
    sigs = {
        "last_error": (C.c_char_p, []),
        "version": (C.c_int, []),
        "struct_sizes": (None, [C.POINTER(C.c_int64)]),
        "scratch_floats": (C.c_int64, [i32, i32]),
        "sim_create": (C.c_int, [C.POINTER(LgxModel), C.POINTER(LgxEnvParams), C.POINTER(LgxBuffers), C.c_int,
                                 C.POINTER(vp)]),
        "sim_destroy": (C.c_int, [vp]),
        "step": (C.c_int, [vp, i64, vp]),
        "simulate": (C.c_int, [vp, i32, vp]),
        "post_physics": (C.c_int, [vp, i64, vp]),
        "post_physics_fused": (C.c_int, [vp, i64, vp]),
        "reset_idx": (C.c_int, [vp, vp, i32, i64, i32, vp]),
        "set_draws": (C.c_int, [vp, vp]),
        "rebind_obs": (C.c_int, [vp, vp]),
        "actuator_mlp": (C.c_int, [vp, vp, i64, vp, vp, vp]),
        "actuator_lstm": (C.c_int, [vp, vp, vp, vp, i64, vp, vp]),
        "mlp_forward": (C.c_int, [vp, vp, i64, i32, C.POINTER(i32), C.POINTER(vp), C.POINTER(vp), i32, vp]),
        "gae": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp]),
        "gae_norm_scratch": (i64, [i32]),
        "gae_norm": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp]),
        "gae_parts": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp]),
        "adv_norm": (C.c_int, [vp, i64, vp, i32, vp]),
        "profile_enable": (C.c_int, [vp, i32]),
        "mlp_forward_batch": (C.c_int, [C.POINTER(LgxMlpDesc), i32, vp]),
        "profile_collect": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    }
    if prefix == "lgx":  # PPO update entry points: product library only
        sigs.update({
            "physics_lane_split": (i32, [i32]),
            "trimesh_build": (C.c_int, [vp, i32, i32, C.c_double, C.c_double, C.c_double, vp, vp, vp, vp]),
            "step_from": (C.c_int, [vp, vp, i64, vp]),
            "drive_inputs": (C.c_int, [vp, vp, vp]),
            "ground_contact": (C.c_int, [vp, vp, i32, vp, vp]),
            "sync_aux": (C.c_int, [vp, vp]),
            "rebind_extras": (C.c_int, [vp, vp]),
            "sim_buffer": (C.c_int, [vp, i32, C.POINTER(vp), C.POINTER(i64), C.POINTER(i32), C.POINTER(i32)]),
            "ppo_gather_rows": (C.c_int, [vp, vp, vp, i64, i32, vp]),
            "ppo_act": (C.c_int, [C.POINTER(LgxPpoActArgs), vp]),
            "ppo_store": (C.c_int, [C.POINTER(LgxPpoStoreArgs), vp]),
            "ppo_act_store": (C.c_int, [C.POINTER(LgxPpoActArgs), C.POINTER(LgxPpoStoreArgs), vp]),
            "bias_act": (C.c_int, [vp, vp, i64, i32, i32, i32, vp]),
            "ppo_loss_partials_floats": (i64, [i64, i32]),
            "ppo_loss": (C.c_int, [C.POINTER(LgxPpoLossArgs), vp]),
            "ppo_adapt_lr": (C.c_int, [vp, C.c_float, vp, C.c_double, vp]),
            "head_bwd_partials_floats": (i64, [i64, i32, i32]),
            "head_bwd": (C.c_int, [vp, vp, vp, vp, vp, i64, i32, i32, vp, vp]),
            "head_bwd_finalize": (C.c_int, [C.POINTER(LgxPpoLossArgs), vp, vp, vp, vp, vp, i64, i32, i32, vp, vp]),
            "colsum_partials_floats": (i64, [i64, i32, i32]),
            "elu_bwd_colsum": (C.c_int, [vp, vp, i64, i32, i32, vp, vp]),
            "reduce_slices": (C.c_int, [C.POINTER(LgxReduceJob), i32, vp]),
            "reduce_slices_finalize": (C.c_int, [C.POINTER(LgxReduceJob), i32, C.POINTER(LgxPpoLossArgs), vp]),
            "reduce_slices_blocks": (i64, [C.POINTER(LgxReduceJob), i32, i32]),
            "reduce_slices_sq": (C.c_int, [C.POINTER(LgxReduceJob), i32, C.POINTER(LgxPpoLossArgs), vp, vp, vp]),
            "ppo_loss_bwd_layout": (C.c_int, [i64, i32, i32, C.POINTER(i64)]),
            "ppo_loss_bwd": (C.c_int, [C.POINTER(LgxPpoLossArgs), vp, vp]),
            "mlp_x3_weight_elems": (i64, [i32, i32]),
            "mlp_x3_split": (C.c_int, [vp, i32, i32, vp, vp]),
            "mlp_x3_split_layers": (C.c_int, [C.POINTER(vp), C.POINTER(i32), i32, C.POINTER(vp), vp]),
            "mlp_x3_lds_bytes": (i64, [C.POINTER(LgxMlpX3Desc), i32]),
            "mlp_x3_forward": (C.c_int, [C.POINTER(LgxMlpX3Desc), i32, vp]),
            "mlp_x3_forward_act": (C.c_int, [C.POINTER(LgxMlpX3Desc), i32, C.POINTER(LgxPpoActArgs),
                                             C.POINTER(LgxPpoStoreArgs), vp]),
            "gemm_partials_floats": (i64, [i64, i32, i32]),
            "gemm_nt": (C.c_int, [C.POINTER(LgxGemmArgs), vp]),
            "gemm_tn": (C.c_int, [C.POINTER(LgxGemmTnArgs), vp]),
            "copy2d": (C.c_int, [C.POINTER(LgxCopy2dJob), i32, vp]),
            "split_bf16_elems": (i64, [i32, i32]),
            "split_bf16": (C.c_int, [C.POINTER(LgxCopy2dJob), i32, vp]),
            "ppo_gather_rows_padded": (C.c_int, [vp, vp, vp, i64, i32, i32, vp]),
            "ppo_gather_rows_padded_dup": (C.c_int, [vp, vp, vp, i64, i32, i32, i64, vp]),
            "adam_clip": (C.c_int, [vp, vp, vp, vp, i64, vp, i32, C.c_float, C.c_float, vp, vp, C.c_float,
                                    C.c_float, C.c_float, vp]),
            "adam_clip_mirror": (C.c_int, [vp, vp, vp, vp, i64, vp, i32, C.c_float, C.c_float, vp, vp, C.c_float,
                                           C.c_float, C.c_float, C.POINTER(LgxCopy2dJob), i32, vp]),
            "adam_clip_mirror_sq": (C.c_int, [vp, vp, vp, vp, i64, vp, i32, C.c_float, vp, vp, C.c_float,
                                              C.c_float, C.c_float, C.POINTER(LgxCopy2dJob), i32, vp]),
            "event_create": (C.c_int, [C.POINTER(vp)]),
            "event_destroy": (C.c_int, [vp]),
            "event_record": (C.c_int, [vp, vp]),
            "stream_wait_event": (C.c_int, [vp, vp]),
            "launch_bind_event": (C.c_int, [vp]),
            "launch_bind_pending": (C.c_int, []),
            "comm_unique_id": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8)]),
            "comm_create": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), i32, i32, i32, C.POINTER(vp)]),
            "comm_destroy": (C.c_int, [vp]),
            "allreduce_grads": (C.c_int, [vp, vp, C.c_size_t, i32, vp]),
        })
    for name, (res, args) in sigs.items():
        fn = getattr(lib, f"{prefix}_{name}")
        fn.restype = res
        fn.argtypes = args
    return lib


EXPORTED = ["lgx_last_error", "lgx_version", "lgx_physics_lane_split", "lgx_trimesh_build", "lgx_struct_sizes", "lgx_scratch_floats", "lgx_sim_create",
            "lgx_sim_destroy", "lgx_step", "lgx_simulate", "lgx_post_physics", "lgx_post_physics_fused", "lgx_reset_idx", "lgx_set_draws", "lgx_rebind_obs", "lgx_rebind_extras", "lgx_sim_buffer", "lgx_step_from", "lgx_drive_inputs", "lgx_ground_contact", "lgx_sync_aux",
            "lgx_actuator_mlp", "lgx_actuator_lstm", "lgx_mlp_forward", "lgx_gae", "lgx_gae_norm_scratch", "lgx_gae_norm", "lgx_gae_parts", "lgx_adv_norm",
            "lgx_profile_enable", "lgx_profile_collect", "lgx_mlp_forward_batch",
            "lgx_ppo_gather_rows", "lgx_bias_act", "lgx_ppo_loss_partials_floats", "lgx_ppo_loss", "lgx_ppo_adapt_lr",
            "lgx_head_bwd_partials_floats", "lgx_head_bwd", "lgx_head_bwd_finalize", "lgx_colsum_partials_floats", "lgx_elu_bwd_colsum",
            "lgx_reduce_slices", "lgx_reduce_slices_finalize", "lgx_ppo_loss_bwd_layout", "lgx_ppo_loss_bwd", "lgx_adam_clip", "lgx_adam_clip_mirror", "lgx_adam_clip_mirror_sq", "lgx_reduce_slices_blocks", "lgx_reduce_slices_sq", "lgx_ppo_act", "lgx_ppo_store", "lgx_ppo_act_store",
            "lgx_gemm_partials_floats", "lgx_gemm_nt", "lgx_copy2d", "lgx_ppo_gather_rows_padded",
            "lgx_ppo_gather_rows_padded_dup", "lgx_split_bf16_elems", "lgx_split_bf16", "lgx_gemm_tn",
            "lgx_mlp_x3_weight_elems", "lgx_mlp_x3_split", "lgx_mlp_x3_split_layers", "lgx_mlp_x3_lds_bytes", "lgx_mlp_x3_forward", "lgx_mlp_x3_forward_act",
            "lgx_event_create", "lgx_event_destroy", "lgx_event_record", "lgx_stream_wait_event",
            "lgx_launch_bind_event", "lgx_launch_bind_pending",
            "lgx_comm_unique_id", "lgx_comm_create", "lgx_comm_destroy", "lgx_allreduce_grads"]


def check_layout(sizes_fn, n=12):
    """Compare the library's sizeof() of every ABI struct with these mirrors (the oracle
    reports the first 3)."""
    out = (C.c_int64 * 16)()
    sizes_fn(out)
    mine = (C.sizeof(LgxModel), C.sizeof(LgxEnvParams), C.sizeof(LgxBuffers), C.sizeof(LgxMlpDesc),
            C.sizeof(LgxPpoLossArgs), C.sizeof(LgxReduceJob), C.sizeof(LgxPpoActArgs),
            C.sizeof(LgxPpoStoreArgs), C.sizeof(LgxGemmArgs), C.sizeof(LgxCopy2dJob), C.sizeof(LgxGemmTnArgs),
            C.sizeof(LgxMlpX3Desc))[:n]
    if tuple(out)[:n] != mine:
        raise RuntimeError(f"lgx ABI layout mismatch: library {tuple(out)[:n]} vs bindings {mine}")
