"""The remaining quadrupeds of the reference registry (legged_gym/envs/__init__.py:52-59):
anymal_b, a1, a1_src, aliengo — built through task_registry on the CPU oracle.

Models are derived from the reference URDFs by tools/urdf_model.py; the totals below are the
URDF link masses summed (collapse_fixed_joints merges, nothing is dropped).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle_backend import make_env

from legged_gym_amd.sim import abi

MASS = {"a1": 12.454, "a1_src": 13.741, "aliengo": 20.638, "anymal_b": 30.6214}
OBS = {"a1": 235, "a1_src": 235, "aliengo": 48, "anymal_b": 235}
EXPERIMENT = {"a1": "rough_a1", "a1_src": "rough_a1_src", "aliengo": "rough_aliengo", "anymal_b": "rough_anymal_b"}


def test_cassie_registry_model_and_config():
    """cassie (envs/__init__.py:54): the reference's biped - 2 legs x 6 revolute joints (leg_dof 6,
    13 bodies named as Isaac Gym names them, the root 'pelvis'), 2 feet ('toe'), pelvis termination by
    substring (pelvis + both *_pelvis_rotation bodies, legged_robot.py:678-680), 169 observations, the
    no_fly term, the reference's gains and default angles (cassie_config.py)."""
    import legged_gym_amd.envs  # noqa: F401
    from legged_gym_amd import LEGGED_GYM_ROOT_DIR
    from legged_gym_amd.utils.task_registry import task_registry
    assert task_registry.task_classes["cassie"].__name__ == "Cassie"
    assert task_registry.train_cfgs["cassie"].runner.experiment_name == "rough_cassie"
    d = json.load(open(os.path.join(LEGGED_GYM_ROOT_DIR, "resources", "cassie_model.json")))
    assert d["leg_dof"] == 6 and len(d["dof_names"]) == 12 and len(d["body_names"]) == 13
    assert d["body_names"][0] == "pelvis" and d["body_names"][6] == "left_toe" and d["body_names"][12] == "right_toe"
    np.testing.assert_allclose(sum(b["mass"] for b in d["dyn_bodies"]), 30.468, rtol=1e-4)   # URDF link masses
    env = make_env("cassie", num_envs=4)
    assert env._lgx_model.leg_dof == 6
    assert env.num_obs == 169 and env.obs_buf.shape == (4, 169) and env.num_height_points == 121
    assert env.feet_indices.tolist() == [6, 12] and env.feet_air_time.shape == (4, 2)
    assert env.termination_contact_indices.tolist() == [0, 1, 7]
    assert "no_fly" in env.reward_names and env.reward_scales["termination"] == pytest.approx(-200 * env.dt)
    assert env.p_gains.tolist() == [100., 100., 200., 200., 200., 40.] * 2
    assert env.default_dof_pos[0].tolist() == pytest.approx([0.1, 0., 1., -1.8, 1.57, -1.57, -0.1, 0., 1., -1.8, 1.57, -1.57])
    env.reset()
    g = torch.Generator().manual_seed(0)
    for _ in range(10):
        obs, _, rew, done, _ = env.step(torch.randn(4, 12, generator=g) * 0.3)
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()


def test_registry_holds_every_quadruped():
    import legged_gym_amd.envs  # noqa: F401
    from legged_gym_amd.utils.task_registry import task_registry
    for name in ("anymal_c_rough", "anymal_c_flat", "anymal_b", "a1", "a1_src", "go1", "aliengo"):
        assert name in task_registry.task_classes
    for name, exp in EXPERIMENT.items():
        assert task_registry.train_cfgs[name].runner.experiment_name == exp
    assert task_registry.task_classes["a1"].__name__ == "LeggedRobot"
    assert task_registry.task_classes["anymal_b"].__name__ == "Anymal"
    assert issubclass(task_registry.task_classes["aliengo"], task_registry.task_classes["go1"])


@pytest.mark.parametrize("task", sorted(MASS))
def test_model_mass_and_layout(task):
    from legged_gym_amd import LEGGED_GYM_ROOT_DIR
    d = json.load(open(os.path.join(LEGGED_GYM_ROOT_DIR, "resources", f"{task}_model.json")))
    assert len(d["dof_names"]) == 12 and len(d["body_names"]) == 17
    total = sum(b["mass"] for b in d["dyn_bodies"])
    np.testing.assert_allclose(total, MASS[task], rtol=1e-4)


@pytest.mark.parametrize("task", sorted(MASS))
def test_steps_on_oracle(task):
    env = make_env(task, num_envs=4)
    env.reset()
    assert env.obs_buf.shape == (4, OBS[task])
    g = torch.Generator().manual_seed(0)
    for _ in range(20):
        obs, _, rew, done, _ = env.step(torch.randn(4, 12, generator=g) * 0.3)
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()


@pytest.mark.parametrize("task,lo,hi", [("a1", 0.24, 0.33), ("anymal_b", 0.40, 0.60)])
def test_pd_standing(task, lo, hi):
    """Zero actions hold the default pose: base height above the terrain under the feet, upright."""
    def ov(c):
        c.domain_rand.push_robots = False
        c.terrain.mesh_type = "plane"
    env = make_env(task, num_envs=2, overrides=ov)
    env.reset()
    for _ in range(100):
        env.step(torch.zeros(2, 12))
    z = env.root_states[:, 2] - env.env_origins[:, 2]
    assert ((z > lo) & (z < hi)).all(), z
    assert (env.projected_gravity[:, 2] < -0.99).all()
    assert not env.reset_buf.any()


def test_anymal_explicit_torques_select_the_sea_network():
    """explicit_torques on ANYmal = the reference's Anymal._compute_torques (anymal.py:71-78): the
    SEA LSTM when use_actuator_network is set (LGX_CTRL_SEA), else LeggedRobot's P / V / T law."""
    from types import SimpleNamespace
    from legged_gym_amd.envs.anymal_c.anymal import Anymal
    ctl = SimpleNamespace(explicit_torques=True, use_actuator_network=True, control_type="P")
    ns = SimpleNamespace(cfg=SimpleNamespace(control=ctl))
    ns._sea_control = lambda: Anymal._sea_control(ns)
    assert Anymal._control_type(ns) == abi.CTRL["SEA"]
    ctl.use_actuator_network = False
    assert Anymal._control_type(ns) == abi.CTRL["P"]
    ctl.explicit_torques, ctl.use_actuator_network = False, True
    assert Anymal._control_type(ns) == abi.CTRL["POS_DRIVE"]
