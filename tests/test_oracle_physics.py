"""Known-answer tests of the lgx physics model on the CPU oracle (PhysX parity is unpinned:
PhysX is closed and absent, so the model is validated against physics it must obey)."""
import numpy as np
import pytest
import torch

from oracle_backend import make_env


def fresh(task="go1_flat_bench", n=4, **cfg):
    def ov(c):
        for k, v in cfg.items():
            obj = c
            *path, last = k.split(".")
            for p in path:
                obj = getattr(obj, p)
            setattr(obj, last, v)
    return make_env(task, num_envs=n, device="cpu", backend="oracle", overrides=ov)


def test_free_fall_is_ballistic():
    env = fresh()
    env.root_states[:, 2] = 5.0                  # far above the ground: no contact
    env.root_states[:, 3:7] = torch.tensor([0, 0, 0, 1.0])
    env.root_states[:, 7:13] = 0
    env.root_states[0, 7] = 1.0                  # initial horizontal velocity
    env.dof_pos[:] = env.default_dof_pos
    env.dof_vel[:] = 0
    env.target_poses[:] = env.default_dof_pos
    dt = env.sim_params.dt
    n = 40
    z0 = env.root_states[:, 2].clone()
    env.simulate(n)
    # semi-implicit Euler: v_n = -g n dt, z_n = z0 - g dt^2 n(n+1)/2 (COM offsets only add tiny internal motion)
    vz = env.root_states[:, 9]
    np.testing.assert_allclose(vz.numpy(), -9.81 * n * dt, rtol=2e-3)
    np.testing.assert_allclose((z0 - env.root_states[:, 2]).numpy(), 9.81 * dt * dt * n * (n + 1) / 2, rtol=2e-2)
    assert abs(env.root_states[0, 7].item() - 1.0) < 1e-2
    assert env.contact_forces.abs().max() == 0


def _rot(axis, th):
    a = np.asarray(axis, np.float64)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _com(env, e):
    """System centre of mass from an independent numpy forward kinematics of the model JSON."""
    d = env.asset.data
    q = env.root_states[e, 3:7].double().numpy()
    x, y, z, w = q
    R0 = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    p0 = env.root_states[e, :3].double().numpy()
    bodies = d["dyn_bodies"]
    tot = bodies[0]["mass"] * (p0 + R0 @ np.array(bodies[0]["com"]))
    msum = bodies[0]["mass"]
    for leg in range(4):
        R, o = R0, p0
        for k in range(3):
            j = 3 * leg + k
            jt = d["joints"][j]
            E = np.array(jt["rot"]).reshape(3, 3)
            o = o + R @ np.array(jt["pos"])
            R = R @ E @ _rot(jt["axis"], env.dof_pos[e, j].item())
            b = bodies[1 + j]
            tot = tot + b["mass"] * (o + R @ np.array(b["com"]))
            msum += b["mass"]
    return tot / msum


def test_centre_of_mass_moves_uniformly_without_external_forces():
    env = fresh(n=2, **{"asset.disable_gravity": True})
    env.body_mass_scale[:] = 1.0
    g = torch.Generator().manual_seed(0)
    env.root_states[:, 2] = 5.0
    env.root_states[:, 7:13] = torch.randn(2, 6, generator=g) * 0.5
    env.dof_pos[:] = env.default_dof_pos + torch.randn(2, 12, generator=g) * 0.2
    env.dof_vel[:] = torch.randn(2, 12, generator=g) * 2
    env.target_poses[:] = env.default_dof_pos     # internal drive forces only
    dt = env.sim_params.dt
    c0 = [_com(env, e) for e in range(2)]
    env.simulate(1)
    c1 = [_com(env, e) for e in range(2)]
    n = 100
    env.simulate(n)
    c2 = [_com(env, e) for e in range(2)]
    for e in range(2):
        v_early = (c1[e] - c0[e]) / dt
        v_late = (c2[e] - c1[e]) / (n * dt)
        # internal forces cannot accelerate the COM (first-order integrator: small drift only)
        np.testing.assert_allclose(v_late, v_early, atol=5e-3 + 0.02 * np.abs(v_early).max())


def test_pd_standing_equilibrium():
    env = fresh(n=2)
    env.reset()
    for _ in range(100):
        env.step(torch.zeros(2, 12))
    z = env.root_states[:, 2]
    assert ((z > 0.25) & (z < 0.36)).all(), z
    fz = env.contact_forces[:, env.feet_indices, 2].sum(1)
    np.testing.assert_allclose(fz.numpy(), 12.013 * 9.81, rtol=0.1)     # feet carry the weight
    assert (env.dof_pos - env.default_dof_pos).abs().max() < 0.15
    assert not env.reset_buf.any()


def test_drive_saturates_at_effort_limit():
    env = fresh(n=2)
    env.reset()
    env.actions[:] = 0
    env.target_poses[:] = env.dof_pos_limits[:, 1]    # far target -> saturated drives
    env.simulate(1)
    assert env.torques.abs().max() <= 23.7 + 1e-4
    assert (env.torques.abs() > 23.0).any()


def test_fallen_robot_terminates():
    env = fresh(n=2)
    env.reset()
    env.root_states[:, 2] = 0.045   # trunk half-height 0.057: corners below ground
    env.root_states[:, 3:7] = torch.tensor([1.0, 0, 0, 0])   # upside down on the trunk
    env.root_states[:, 7:] = 0
    env.simulate(4)
    assert (env.contact_forces[:, 0].norm(dim=-1) > 1.0).all()


def test_rough_terrain_contact_follows_heightfield():
    env = fresh("go1_rough", n=8)
    env.reset()
    for _ in range(30):
        env.step(torch.zeros(8, 12))
    # robots stand on the terrain: base height above local ground in a sane band
    hs = env.height_samples
    ij = ((env.root_states[:, :2] + env.cfg.terrain.border_size) / env.cfg.terrain.horizontal_scale).long()
    ground = hs[ij[:, 0], ij[:, 1]].float() * env.cfg.terrain.vertical_scale
    h = env.root_states[:, 2] - ground
    assert torch.isfinite(env.root_states).all()
    assert (h > 0.0).float().mean() > 0.8


def test_returned_obs_survive_the_next_step():
    """The reference returns a fresh obs tensor every step (legged_robot.py:218); rsl_rl stores the
    transition's obs after the following env.step, so that tensor must not be overwritten."""
    env = fresh(n=4)
    env.reset()
    obs0, *_ = env.step(torch.zeros(4, 12))
    keep = obs0.clone()
    obs1, *_ = env.step(torch.ones(4, 12) * 0.3)
    assert obs1.data_ptr() != obs0.data_ptr()
    assert torch.equal(obs0, keep)
    assert torch.equal(env.get_observations(), obs1)
