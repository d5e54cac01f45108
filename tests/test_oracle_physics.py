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


@pytest.mark.parametrize("task", ["go1_flat_bench", "cassie"])
def test_free_fall_is_ballistic(task):
    env = fresh(task, **{"terrain.mesh_type": "plane"})
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
    LD = d.get("leg_dof", 3)
    tot = bodies[0]["mass"] * (p0 + R0 @ np.array(bodies[0]["com"]))
    msum = bodies[0]["mass"]
    for leg in range(12 // LD):
        R, o = R0, p0
        for k in range(LD):
            j = LD * leg + k
            jt = d["joints"][j]
            E = np.array(jt["rot"]).reshape(3, 3)
            o = o + R @ np.array(jt["pos"])
            R = R @ E @ _rot(jt["axis"], env.dof_pos[e, j].item())
            b = bodies[1 + j]
            tot = tot + b["mass"] * (o + R @ np.array(b["com"]))
            msum += b["mass"]
    return tot / msum


@pytest.mark.parametrize("task", ["go1_flat_bench", "cassie"])
def test_centre_of_mass_moves_uniformly_without_external_forces(task):
    """Momentum conservation: internal drive forces cannot accelerate the centre of mass, for the
    quadruped (4 x 3 joint chains) and the biped (2 x 6)."""
    env = fresh(task, n=2, **{"asset.disable_gravity": True, "terrain.mesh_type": "plane"})
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


def _pendulum_period(lib_simulate, kp, steps=700):
    """Calf joint of leg 0 as a torsional pendulum: no gravity, the base made 1e6x heavier (a fixed
    pivot), hip / thigh held by stiff implicit drives, the calf's implicit position drive with
    stiffness kp and no damping as the spring.  Returns (measured period, discrete-map period,
    continuous period 2 pi sqrt(I / kp)) in seconds."""
    env = fresh(n=2)
    m = env._backend.m
    dt = float(m.sim_dt)
    m.gravity[0] = m.gravity[1] = m.gravity[2] = 0.0
    j = 2                                          # FL calf; dynamic body 1 + j
    b = 1 + j
    for k in range(12):
        m.kp[k], m.kd[k] = (kp, 0.0) if k == j else (1e5, 50.0)
    env.body_mass_scale[:, 0] = 1e6
    env.root_states[:, :3] = torch.tensor([0.0, 0.0, 5.0])
    env.root_states[:, 3:7] = torch.tensor([0, 0, 0, 1.0])
    env.root_states[:, 7:] = 0
    env.dof_pos[:] = env.default_dof_pos
    env.dof_vel[:] = 0
    env.target_poses[:] = env.default_dof_pos
    th0 = float(env.default_dof_pos[0, j])
    env.dof_pos[:, j] = th0 + 0.1
    # effective inertia about the joint axis: axis^T I_com axis + m |axis x com|^2 (body frame)
    a = np.array(m.joint_axis[j][:], np.float64)
    I6 = np.array(m.body_inertia[b][:], np.float64)
    Ib = np.array([[I6[0], I6[3], I6[4]], [I6[3], I6[1], I6[5]], [I6[4], I6[5], I6[2]]])
    c = np.array(m.body_com[b][:], np.float64)
    I_eff = a @ Ib @ a + float(m.body_mass[b]) * (c @ c - (a @ c) ** 2)
    k = float(np.float32(kp)) / I_eff
    # implicit drive, kd = 0: (I + dt^2 kp) v' = I v - dt kp th, th' = th + dt v' 
    al = 1.0 / (1.0 + dt * dt * k)
    trace, det = 1.0 + al * (1.0 - dt * dt * k), al
    phi = np.arccos(trace / (2.0 * np.sqrt(det)))
    t_disc, t_cont = 2 * np.pi * dt / phi, 2 * np.pi / np.sqrt(k)
    th = []
    for _ in range(steps):
        lib_simulate(env, 1)
        th.append(float(env.dof_pos[0, j]) - th0)
    th = np.array(th)
    ups = [i + th[i] / (th[i] - th[i + 1]) for i in range(len(th) - 1) if th[i] < 0 <= th[i + 1]]
    assert len(ups) >= 3, ups
    t_meas = (ups[-1] - ups[0]) / (len(ups) - 1) * dt
    return t_meas, t_disc, t_cont


@pytest.mark.parametrize("build", ["f32", "f64"])
def test_pendulum_period(build):
    """SURVEY.md 8(c) known answer: a one-joint torsional pendulum oscillates with the period of
    the integrator's own map (1e-4 in float32, 5e-5 in float64; measured 7e-6 - the residual is the
    coupling to the stiffly held joints and the 1e6x base) and within 0.5 % of the continuous
    2 pi sqrt(I / kp) (implicit Euler's phase lag: 0.13 % at omega dt = 0.063)."""
    from oracle_backend import simulate64
    sim = (lambda env, n: env.simulate(n)) if build == "f32" else simulate64
    kp = 1.2
    t_meas, t_disc, t_cont = _pendulum_period(sim, kp)
    assert 0.3 < t_cont < 3.0, t_cont
    tol = 1e-4 if build == "f32" else 5e-5
    assert abs(t_meas / t_disc - 1) < tol, (t_meas, t_disc)
    assert abs(t_meas / t_cont - 1) < 5e-3, (t_meas, t_cont)


def test_float64_oracle_bounds_float32_error():
    """The float64 physics build agrees with the float32 one to float32 rounding through the
    ill-conditioned implicit solve (one env step = 4 substeps, rough terrain, 64 envs): velocities
    to 2e-3 relative to their scale, contact forces to 0.05 N, and the two builds are not identical
    (it is a different arithmetic, not a copy)."""
    from oracle_backend import simulate64
    from test_gpu_parity import randomize_state
    env = make_env("go1_rough", num_envs=64, device="cpu", backend="oracle")
    g = torch.Generator().manual_seed(3)
    randomize_state(env, g)
    s0 = {k: getattr(env, k).clone() for k in ("root_states", "dof_state")}
    env.simulate(4)
    f32 = (env.root_states.clone(), env.dof_state.clone(), env.contact_forces.clone())
    env.root_states.copy_(s0["root_states"])
    env.dof_state.copy_(s0["dof_state"])
    simulate64(env, 4)
    f64 = (env.root_states.clone(), env.dof_state.clone(), env.contact_forces.clone())
    for a, b, tol in zip(f32, f64, (2e-3, 2e-3, 0.05)):
        d = (a - b).abs().max().item()
        assert 0 < d <= tol * max(1.0, b.abs().max().item() if tol < 0.01 else 1.0), d
