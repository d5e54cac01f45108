"""Oracle vs the reference's own Python: golden-vector replay (CPU).

tests/golden/*.npz were produced by tools/golden/gen_golden.py, which ran the reference's
`LeggedRobot`/`Go1`/`Anymal` post-physics code (legged_robot.py:79-231, 337-463, 818-966;
go1.py:79-107) with scripted physics outputs and an injected draw table.  Here the SAME
inputs (initial state, actions, scripted physics state, draw table) are replayed through the
lgx host setup + CPU oracle and every output is compared.

Tolerances: float32 arithmetic on both sides with different summation orders (torch
reductions vs sequential C): obs/commands/state 2e-5 abs + 1e-5 rel; rewards and episode sums
1e-5 abs + 1e-4 rel; booleans, episode lengths and terrain levels exact.
"""
import os

import numpy as np
import pytest
import torch

from oracle_backend import load_oracle, make_env, vp

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = {"go1_flat": "go1", "go1_rough": "go1_rough", "anymal_c_rough": "anymal_c_rough",
         # 24 envs x 36 steps on other seeds / terrain draws (the short cases: 12-24 envs x 12-24)
         "go1_rough_long": "go1_rough", "anymal_c_rough_long": "anymal_c_rough",
         # the biped (envs/cassie: 2 feet, _reward_no_fly, 11 x 11 scan, pelvis termination)
         "cassie_rough": "cassie"}


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))


def build(name, g, device="cpu", backend="oracle", overrides=None):
    env = make_env(CASES[name], num_envs=int(g["num_envs"]), device=device, backend=backend, overrides=overrides)
    if "height_samples" in g:
        assert tuple(env.height_samples.shape) == g["height_samples"].shape
        env.height_samples.copy_(torch.from_numpy(g["height_samples"]))
        env.terrain_origins.copy_(torch.from_numpy(g["terrain_origins"]))
        env.terrain_types.copy_(torch.from_numpy(g["terrain_types"]))
    st = lambda k: torch.from_numpy(np.asarray(g["init_" + k])).to(device)
    env.root_states.copy_(st("root_states"))
    env.dof_state.copy_(st("dof_state"))
    env.commands.copy_(st("commands"))
    env.feet_air_time.copy_(st("feet_air_time"))
    env._episode_length_buf.copy_(st("episode_length_buf"))
    env.last_actions.copy_(st("last_actions"))
    env.last_dof_vel.copy_(st("last_dof_vel"))
    env.last_root_vel.copy_(st("last_root_vel"))
    env.env_origins.copy_(st("env_origins"))
    env.actions.copy_(st("last_actions"))
    if "init_terrain_levels" in g:
        env.terrain_levels.copy_(st("terrain_levels"))
    rows = env.reward_names + (["termination"] if "termination" in env.reward_scales else [])
    init = st("episode_sums")
    for i, k in enumerate(env.episode_sums):     # golden rows are in dict key order
        env._episode_sums_buf[rows.index(k)].copy_(init[i])
    if "init_act_hist" in g:
        env.actuator_history.copy_(st("act_hist").reshape(env.num_envs, -1))
    env.common_step_counter = int(g["init_common_step_counter"])
    return env


def sums_by_key(env, buf=None):
    """Episode sums stacked in the env's dict key order (the reference's: the golden's rows)."""
    buf = env._episode_sums_buf if buf is None else buf
    rows = env.reward_names + (["termination"] if "termination" in env.reward_scales else [])
    return buf[[rows.index(k) for k in env.episode_sums]]


def extras_by_key(env):
    """extras["episode"] reward means in the env's dict key order (the golden's rows)."""
    rows = dict(env._extras_rows)
    return env._extras_buf[[rows["rew_" + k] for k in env.episode_sums]]


def close(a, b, atol, rtol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    return err.max() <= 0, float(np.abs(a - b).max())


@pytest.mark.parametrize("name", list(CASES))
def test_setup_constants_match_reference(name):
    g = load(name)
    env = make_env(CASES[name], num_envs=int(g["num_envs"]), device="cpu", backend="oracle", seed=int(g["seed"]))
    assert env.max_episode_length == float(g["max_episode_length"]) == 1001.0       # legged_robot.py:777
    assert env.dt == pytest.approx(float(g["dt"]), abs=0)
    assert env.cfg.domain_rand.push_interval == float(g["push_interval"])
    assert list(env.reward_names) == [str(x) for x in g["reward_names"]]            # alphabetical order
    np.testing.assert_allclose([env.reward_scales[k] for k in env.reward_names], g["reward_scales"], rtol=1e-12)
    np.testing.assert_allclose(env.noise_scale_vec.numpy(), g["noise_scale_vec"], rtol=1e-7)
    np.testing.assert_allclose(env.dof_pos_limits.numpy(), g["dof_pos_limits"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(env.default_dof_pos.numpy(), g["default_dof_pos"])
    assert env.feet_indices.tolist() == g["feet_indices"].tolist()
    assert env.penalised_contact_indices.tolist() == g["penalised_contact_indices"].tolist()
    assert env.termination_contact_indices.tolist() == g["termination_contact_indices"].tolist()
    assert list(env.episode_sums.keys()) == [str(x) for x in g["episode_keys"]]
    # domain randomisation at creation (legged_robot.py:259-335) with the same seed: friction
    # buckets (CPU torch generator) and per-env body masses (numpy) as the reference set them
    if "dr_friction" in g:
        np.testing.assert_array_equal(env.friction_coeffs.numpy(), g["dr_friction"])
    np.testing.assert_allclose(env.body_masses, g["dr_body_masses"], rtol=1e-12, atol=0)
    # terrain placement at creation (legged_robot.py:742-767): levels, types -> env origins
    if "setup_terrain_levels" in g:
        np.testing.assert_array_equal(env.terrain_levels.numpy(), g["setup_terrain_levels"])
    np.testing.assert_allclose(env.env_origins.numpy(), g["setup_env_origins"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", list(CASES))
def test_post_physics_replay_matches_reference(name):
    g = load(name)
    env = build(name, g)
    lib = load_oracle()
    be = env._backend
    N, T = int(g["num_envs"]), int(g["steps"])
    dec = env.cfg.control.decimation
    for t in range(T):
        # LeggedRobot.step with the physics replaced by the recorded (scripted) outputs
        env.actions.copy_(torch.clamp(torch.from_numpy(g["step_actions"][t]), -env.cfg.normalization.clip_actions,
                                      env.cfg.normalization.clip_actions))
        lib.lgxo_compute_targets(*be._args())
        for s in range(dec):
            if env._lgx_params.use_actuator_history:
                lib.lgxo_actuator_history(*be._args(), s)
        env.root_states.copy_(torch.from_numpy(g["step_next_root"][t]))
        env.dof_state.copy_(torch.from_numpy(g["step_next_dof"][t]))
        env._contact_forces_full.copy_(torch.from_numpy(g["step_next_cf"][t]).view(N, -1, 3))
        env.torques.copy_(torch.from_numpy(g["step_next_tq"][t]).view(N, -1))
        draws = torch.from_numpy(g["step_draws"][t]).contiguous()
        be.set_draws(draws)
        env.post_physics_step()
        be.set_draws(None)
        tag = f"{name} step {t}"
        np.testing.assert_array_equal(env.reset_buf.numpy(), g["step_reset_buf"][t], err_msg=tag + " reset")
        np.testing.assert_array_equal(env.time_out_buf.numpy(), g["step_time_out_buf"][t], err_msg=tag + " time_out")
        np.testing.assert_array_equal(env._episode_length_buf.numpy(), g["step_episode_length_buf"][t], err_msg=tag)
        for key, mine, tol in (("obs_buf", env.obs_buf, (2e-5, 1e-5)), ("commands", env.commands, (2e-5, 1e-5)),
                               ("root_states", env.root_states, (2e-5, 1e-6)), ("dof_state", env.dof_state, (2e-5, 1e-6)),
                               ("feet_air_time", env.feet_air_time, (1e-6, 1e-6)),
                               ("last_actions", env.last_actions, (0, 0)), ("last_dof_vel", env.last_dof_vel, (0, 0)),
                               ("last_root_vel", env.last_root_vel, (0, 0)), ("base_lin_vel", env.base_lin_vel, (1e-6, 1e-6)),
                               ("base_ang_vel", env.base_ang_vel, (1e-6, 1e-6)),
                               ("projected_gravity", env.projected_gravity, (1e-6, 1e-6)),
                               ("env_origins", env.env_origins, (0, 0)), ("target_poses", env.target_poses, (1e-6, 1e-6)),
                               ("rew_buf", env.rew_buf, (1e-5, 1e-4)),
                               ("episode_sums", sums_by_key(env), (1e-5, 1e-4))):
            ok, err = close(mine.numpy(), g["step_" + key][t], *tol)
            assert ok, f"{tag} {key} max err {err}"
        if "height_samples" in g:
            ok, err = close(env.measured_heights.numpy(), g["step_measured_heights"][t], 1e-6, 0)
            assert ok, f"{tag} heights max err {err}"
            np.testing.assert_array_equal(env.terrain_levels.numpy(), g["step_terrain_levels"][t], err_msg=tag)
        if env._lgx_params.use_actuator_history:
            ok, err = close(env.model_ins.numpy(), g["step_model_ins"][t], 1e-6, 1e-6)
            assert ok, f"{tag} model_ins max err {err}"
        ref_ex = g["step_extras"][t]
        if not np.isnan(ref_ex[0]):   # the reference publishes extras only when an env reset
            T_rows = len(env.episode_sums)
            ok, err = close(extras_by_key(env).numpy(), ref_ex[:T_rows], 1e-6, 1e-4)
            assert ok, f"{tag} extras max err {err}"
            if env.cfg.terrain.curriculum:
                ok, err = close(env._extras_buf.numpy()[T_rows], ref_ex[-1], 1e-6, 1e-6)
                assert ok, f"{tag} terrain_level extras err {err}"
        np.testing.assert_array_equal(env._extras_time_outs.numpy(), g["step_extras_time_outs"][t], err_msg=tag)


GO1_CASES = [n for n in CASES if CASES[n].startswith("go1")]
SEA_CASES = [n for n in CASES if CASES[n].startswith("anymal")]


def sea_control(cfg):
    """ANYmal's SEA network as the step's torque source (LGX_CTRL_SEA, anymal.py:71-77)."""
    cfg.control.explicit_torques = True


@pytest.mark.parametrize("name", GO1_CASES)
def test_go1_actuator_dvel_matches_reference(name):
    """The Go1 actuator-net OUTPUT against the reference's own wrapper code: dVel of every substep
    as go1.py's actuator_advance computed it (UniNet leg slicing, go1.py:22-35; dVel *= vel_std,
    :100-105) around go1_net.pt's MLP rebuilt from its weights (tools/golden/gen_golden.py), vs the
    oracle's history (lgxo_drive_inputs) + UniNet restatement (lgxo_actuator_mlp).  Float32 MLP
    on both sides (different summation order): 2e-5 abs + 1e-5 rel."""
    g = load(name)
    assert "step_dvel" in g
    env = build(name, g)
    lib = load_oracle()
    be = env._backend
    T, dec = int(g["steps"]), env.cfg.control.decimation
    clip = env.cfg.normalization.clip_actions
    for t in range(T):
        env.actions.copy_(torch.clamp(torch.from_numpy(g["step_actions"][t]), -clip, clip))
        lib.lgxo_drive_inputs(*be._args())
        rows = env._model_ins_all.numel() // 30
        lib.lgxo_actuator_mlp(vp(env._model_ins_all), vp(env._actuator_dvel), rows, vp(be._act_w),
                              vp(env.actuator_net_scale))
        assert env._actuator_dvel.shape == g["step_dvel"][t].shape == (dec, int(g["num_envs"]), 12)
        ok, err = close(env._actuator_dvel.numpy(), g["step_dvel"][t], 2e-5, 1e-5)
        assert ok, f"{name} step {t}: dVel max err {err}"
        # the next step's history reads the post-step (post-reset) state of the scripted physics
        env.dof_state.copy_(torch.from_numpy(g["step_dof_state"][t]))


@pytest.mark.parametrize("name", SEA_CASES)
def test_sea_actuator_net_matches_reference(name):
    """The ANYmal SEA torque path against the reference's own `_compute_torques` (anymal.py:71-77,
    called `decimation` times per step on the pre-step state by tools/golden/gen_golden.py around
    anydrive_v3_lstm.pt's LSTMsea rebuilt from its weights) and `reset_idx`'s state zeroing
    (anymal.py:56-60): per step the oracle's drive inputs (lgxo_drive_inputs: 4 LSTM steps) from the
    reference's previous LSTM state -> the last substep's torques (clamped to the drive's effort
    limit, PhysX effort mode) and the state of the envs that do not reset; then the scripted
    post-physics step -> the state of every env, zero for the envs that reset."""
    g = load(name)
    env = build(name, g, overrides=sea_control)
    from legged_gym_amd.sim import abi
    assert env._lgx_params.control_type == abi.CTRL["SEA"]
    lib = load_oracle()
    be = env._backend
    N, T = int(g["num_envs"]), int(g["steps"])
    clip = env.cfg.normalization.clip_actions
    eff = env.torque_limits.numpy()
    for t in range(T):
        tag = f"{name} step {t}"
        env.sea_hidden_state.copy_(torch.from_numpy(g["init_sea_h"] if t == 0 else g["step_sea_h"][t - 1]))
        env.sea_cell_state.copy_(torch.from_numpy(g["init_sea_c"] if t == 0 else g["step_sea_c"][t - 1]))
        env.actions.copy_(torch.clamp(torch.from_numpy(g["step_actions"][t]), -clip, clip))
        lib.lgxo_drive_inputs(*be._args())
        want = np.clip(g["step_sea_torques"][t][-1], -eff, eff)
        ok, err = close(env.torques.numpy(), want, 1e-4, 1e-5)
        assert ok, f"{tag} SEA torques max err {err}"
        keep = ~g["step_reset_buf"][t].astype(bool)
        for mine, key in ((env.sea_hidden_state, "step_sea_h"), (env.sea_cell_state, "step_sea_c")):
            ok, err = close(mine.numpy().reshape(2, N, 12, 8)[:, keep], g[key][t].reshape(2, N, 12, 8)[:, keep],
                            1e-5, 1e-5)
            assert ok, f"{tag} {key} (4 LSTM steps) max err {err}"
        env.root_states.copy_(torch.from_numpy(g["step_next_root"][t]))
        env.dof_state.copy_(torch.from_numpy(g["step_next_dof"][t]))
        env._contact_forces_full.copy_(torch.from_numpy(g["step_next_cf"][t]).view(N, -1, 3))
        env.torques.copy_(torch.from_numpy(g["step_next_tq"][t]).view(N, -1))
        be.set_draws(torch.from_numpy(g["step_draws"][t]).contiguous())
        env.post_physics_step()
        be.set_draws(None)
        np.testing.assert_array_equal(env.reset_buf.numpy(), g["step_reset_buf"][t], err_msg=tag + " reset")
        for mine, key in ((env.sea_hidden_state, "step_sea_h"), (env.sea_cell_state, "step_sea_c")):
            ok, err = close(mine.numpy(), g[key][t], 1e-5, 1e-5)
            assert ok, f"{tag} {key} after reset_idx max err {err}"
            assert (mine.numpy().reshape(2, N, 12, 8)[:, ~keep] == 0).all(), tag
