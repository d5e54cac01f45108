"""GPU parity: the HIP product path (liblgx.so via the C-ABI) against the CPU oracle.

Every test builds the same task twice through the same host setup — once with the oracle
backend on CPU tensors, once with the product backend on cuda:0 — puts both into the same
state and compares outputs.  Tolerances (float32; the oracle uses a different formulation
of the dynamics — dense 18x18 Cholesky vs the kernel's per-leg Schur complement — so
agreement is to rounding, not bitwise):
  physics state after 4 substeps: derived from the float64 build of the oracle's physics
  (check_derived: per-env HIP error vs float64 against the float32 oracle's error vs float64,
  worst env and 90th percentile, see PHYS_C_MAX / PHYS_C_Q90); multi-step / env-logic
  comparisons keep fixed bounds:
  |d| <= 2e-3 + 2e-3 |x| (velocities), 1e-4 (positions)
  env logic with identical inputs: obs/rew 1e-4 abs; integer/bool outputs exact.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle_backend import OracleBackend, make_env, load_oracle, uninet_torch_layout

pytestmark = pytest.mark.gpu

STATE = ["root_states", "dof_state", "target_poses", "torques", "_contact_forces_full", "actions", "last_actions",
         "last_dof_vel", "last_root_vel", "commands", "feet_air_time", "_episode_length_buf", "_episode_sums_buf",
         "env_origins", "terrain_levels", "body_mass_scale", "friction_coeffs", "reset_buf", "time_out_buf",
         "measured_heights"]


def sync(src, dst):
    for name in STATE:
        s, d = getattr(src, name), getattr(dst, name)
        d.copy_(s.to(d.device))
    if hasattr(src, "actuator_history"):
        dst.actuator_history.copy_(src.actuator_history.to(dst.device))


def randomize_state(env, gen, standing=True):
    N = env.num_envs
    r = lambda *s: torch.rand(*s, generator=gen)
    rs = env.root_states
    rs[:, :2] = env.env_origins[:, :2] + (r(N, 2) - 0.5)
    rs[:, 2] = env.env_origins[:, 2] + (0.25 + 0.15 * r(N) if standing else 0.05 + 0.5 * r(N))
    q = torch.randn(N, 4, generator=gen) * torch.tensor([0.15, 0.15, 1.0, 0.0]) + torch.tensor([0, 0, 0, 1.0])
    rs[:, 3:7] = q / q.norm(dim=1, keepdim=True)
    rs[:, 7:13] = (r(N, 6) - 0.5) * 1.0
    env.dof_pos[:] = env.default_dof_pos + (r(N, 12) - 0.5) * 0.6
    env.dof_vel[:] = (r(N, 12) - 0.5) * 4.0
    env.actions[:] = (r(N, 12) - 0.5) * 3.0
    env.target_poses[:] = torch.clip(env.actions * env.cfg.control.action_scale + env.default_dof_pos,
                                     env.dof_pos_limits[:, 0], env.dof_pos_limits[:, 1])
    env.commands[:, :3] = (r(N, 3) - 0.5) * 2
    env.commands[:, 3] = (r(N) - 0.5) * 6
    env.last_actions[:] = (r(N, 12) - 0.5)
    env.last_dof_vel[:] = (r(N, 12) - 0.5)
    env._episode_length_buf[:] = torch.randint(0, 1002, (N,), generator=gen)


def close(a, b, atol, rtol=0.0):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    err = (a - b).abs() - (atol + rtol * b.abs())
    return err.max().item() <= 0, (a - b).abs().max().item()


@pytest.fixture(scope="module")
def envs_flat(gpu):
    ora = make_env("go1_flat_bench", num_envs=64, device="cpu", backend="oracle")
    dev = make_env("go1_flat_bench", num_envs=64, device="cuda:0", backend="lgx")
    return ora, dev


def test_library_loaded_is_in_tree(gpu, envs_flat):
    from legged_gym_amd.sim import lib
    assert lib._LIB is not None and lib.LIB_PATH.endswith("legged_gym_amd/liblgx.so")


# Physics tolerances are DERIVED from a float64 truth (oracle/liblgx_oracle64.so: the oracle's
# physics in double precision from the same start state), per env (an env's error = its largest
# element error of the quantity):
#   * the worst env of the HIP kernel within PHYS_C_MAX x the float32 oracle's worst env, and its
#     90th-percentile env within PHYS_C_Q90 x the oracle's, each plus a floor of PHYS_ULPS float32
#     ulps of the quantity's scale (where the float32 oracle happens to be exact);
#   * an env above the worst-env bound must be EXPLAINED by a branch flip: the contact model is
#     discontinuous (drive saturation, joint limits, a candidate touching or not, stick / slide /
#     separate), and a state within rounding of such a threshold can take either branch in float32.
#     The float64 run records every decision with its relative distance to the threshold; the
#     outlier env's nearest decisions (|margin| <= BRANCH_MARGIN_MAX) are flipped one at a time, and
#     two at a time, in forced float64 runs, and the env must come within the bound of one of those
#     branch truths in EVERY quantity (explain_outliers; the flip and its margin are recorded in
#     BRANCH_FLIPS).  An outlier that no near-threshold flip explains fails the test.
# The two float32 paths use different algorithms (dense 18x18 Cholesky vs per-leg Schur complement
# with fma contraction), so their rounding differs: measured worst-env ratios 0.4-9x over 24
# randomised 64-env states (standing and falling), 90th-percentile ratios <= 3x.
PHYS_C_MAX = 16.0
PHYS_C_Q90 = 4.0
PHYS_ULPS = 64
BRANCH_MARGIN_MAX = 1e-3      # relative distance to a decision's threshold that float32 rounding can cross
BRANCH_CANDIDATES = 12        # nearest decisions tried per outlier env (single flips; pairs among the first 6)
BRANCH_FLIPS = []             # (quantity set, env, flips, margins, HIP error before / after) of explained outliers
PHYS_QTY = {"root_pose": lambda e: e.root_states[:, :7], "root_vel": lambda e: e.root_states[:, 7:],
            "dof_pos": lambda e: e.dof_pos, "dof_vel": lambda e: e.dof_vel, "torques": lambda e: e.torques,
            "contact_forces": lambda e: e.contact_forces}
PHYS_STATE = ("root_states", "dof_state", "torques", "_contact_forces_full")


class Float64Truth(dict):
    """{quantity: float64 tensor} after `n` float64 substeps from an oracle env's state, with what
    a forced re-run needs: the start state and the recorded decisions."""

    def forced(self, flips):
        """The float64 quantities of a run from the same start state with `flips` (env, substep,
        kind, index, decision) taken; the oracle env's current state is restored afterwards."""
        from oracle_backend import simulate64
        ora = self.ora
        cur = {k: getattr(ora, k).clone() for k in PHYS_STATE}
        for k, v in self.s0.items():
            getattr(ora, k).copy_(v)
        simulate64(ora, self.n, force=flips)
        out = {k: f(ora).detach().double().clone() for k, f in PHYS_QTY.items()}
        for k, v in cur.items():
            getattr(ora, k).copy_(v)
        return out


def float64_truth(ora, n, state=PHYS_STATE):
    """Float64Truth after `n` substeps of the float64 physics from the oracle env's current state
    (decisions recorded); the oracle env's state is restored afterwards."""
    from oracle_backend import simulate64
    s0 = {k: getattr(ora, k).clone() for k in state}
    rec = simulate64(ora, n, record=True)
    out = Float64Truth({k: f(ora).detach().double().clone() for k, f in PHYS_QTY.items()})
    for k, v in s0.items():
        getattr(ora, k).copy_(v)
    out.ora, out.n, out.s0, out.records = ora, n, s0, rec
    return out


def _env_errors(truth, hip_vals, e, qty):
    return {k: (hip_vals[k][e].detach().cpu().double() - truth[k][e]).abs().max().item() for k in qty}


def explain_outliers(t64, hip_vals, envs, bounds, qty):
    """Every env in `envs` (original indices) above its worst-env bound in some quantity must come
    within `bounds` in every quantity of `qty` against the float64 truth of a near-threshold branch
    flip (one, or two among the nearest); returns [(env, flips, margins)], appends to BRANCH_FLIPS."""
    from oracle_backend import BRANCH_ALTERNATIVES, BRANCH_KINDS
    import itertools
    out = []
    for e in envs:
        before = _env_errors(t64, hip_vals, e, qty)
        near = sorted((r for r in t64.records if r[0] == e and abs(r[5]) <= BRANCH_MARGIN_MAX), key=lambda r: abs(r[5]))
        near = near[:BRANCH_CANDIDATES]
        singles = [[(r, alt)] for r in near for alt in BRANCH_ALTERNATIVES[r[2]] if alt != r[4]]
        pairs = [a + b for a, b in itertools.combinations(
            [[(r, alt)] for r in near[:6] for alt in BRANCH_ALTERNATIVES[r[2]] if alt != r[4]], 2)
            if a[0][0] is not b[0][0]]
        found = None
        for cand in singles + pairs:
            flips = [(r[0], r[1], r[2], r[3], alt) for r, alt in cand]
            errs = _env_errors(t64.forced(flips), hip_vals, e, qty)
            if all(errs[k] <= bounds[k] for k in qty):
                found = (flips, [r[5] for r, _ in cand], errs)
                break
        assert found is not None, (
            f"env {e}: HIP error vs float64 above the worst-env bound ({before}, bounds {bounds}) and no flip of its "
            f"{len(near)} decisions within {BRANCH_MARGIN_MAX} of a threshold explains it; nearest decisions: "
            f"{[(BRANCH_KINDS[r[2]], r[1], r[3], r[4], r[5]) for r in sorted((r for r in t64.records if r[0] == e), key=lambda r: abs(r[5]))[:5]]}")
        flips, margins, errs = found
        desc = [(BRANCH_KINDS[f[2]], f"substep {f[1]}", f"index {f[3]}", f"-> {f[4]}") for f in flips]
        BRANCH_FLIPS.append({"env": e, "flips": desc, "margins": margins, "hip_err_before": before,
                             "hip_err_on_flipped_branch": errs})
        out.append((e, flips, margins))
    return out


def check_derived(t64, ora_vals, hip_vals, keep=None, qty=None):
    """The derived physics tolerance above for every quantity (rows `keep` only when given), with
    every env above the worst-env bound explained by a branch flip (explain_outliers).
    Returns {quantity: (HIP worst-env error, oracle worst-env error)}."""
    out, bounds, outliers = {}, {}, set()
    qty = list(qty or PHYS_QTY)
    n_all = t64[qty[0]].shape[0]
    idx = torch.arange(n_all) if keep is None else torch.arange(n_all)[keep]
    for k in qty:
        t, o, h = t64[k], ora_vals[k].detach().cpu().double(), hip_vals[k].detach().cpu().double()
        if keep is not None:
            t, o, h = t[keep], o[keep], h[keep]
        n = t.shape[0]
        eh = (h - t).abs().reshape(n, -1).max(1).values
        eo = (o - t).abs().reshape(n, -1).max(1).values
        floor = PHYS_ULPS * 2.0 ** -23 * t.abs().max().item()
        bounds[k] = PHYS_C_MAX * eo.max().item() + floor
        outliers |= set(idx[eh > bounds[k]].tolist())
        qh, qo = torch.quantile(eh, 0.9).item(), torch.quantile(eo, 0.9).item()
        assert qh <= PHYS_C_Q90 * qo + floor, f"{k}: 90th-percentile env error {qh:.3g} > {PHYS_C_Q90} x {qo:.3g} + {floor:.3g}"
        out[k] = (eh.max().item(), eo.max().item())
    if outliers:   # (hip_vals rows are numbered like the truth's envs; keep only selects among them)
        explain_outliers(t64, hip_vals, sorted(outliers), bounds, qty)
    return out


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_physics_substeps_match_oracle(envs_flat, seed):
    """4 physics substeps from randomised states (standing / falling), HIP vs the float64 truth
    with the derived tolerance (check_derived), plus the float32 oracle directly at the old
    fixed bounds."""
    ora, dev = envs_flat
    gen = torch.Generator().manual_seed(seed)
    randomize_state(ora, gen, standing=seed % 2 == 0)
    sync(ora, dev)
    t64 = float64_truth(ora, 4)
    ora.simulate(4)
    dev.simulate(4)
    torch.cuda.synchronize()
    check_derived(t64, {k: f(ora) for k, f in PHYS_QTY.items()}, {k: f(dev) for k, f in PHYS_QTY.items()})
    ok, e = close(dev.root_states[:, 7:], ora.root_states[:, 7:], 2e-3, 2e-3)
    assert ok, f"root vel max err {e}"
    ok, e = close(dev.contact_forces, ora.contact_forces, 0.05, 5e-3)
    assert ok, f"contact force max err {e}"


@pytest.mark.parametrize("task", ["go1_rough", "anymal_c_rough"])
def test_physics_rough_terrain_derived_tolerance(gpu, task):
    """The rough-terrain physics (slope-corrected trimesh contact, 37-92 candidates) against the
    float64 truth with the derived tolerance, 3 seeds."""
    ora = make_env(task, num_envs=64, device="cpu", backend="oracle")
    dev = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    for seed in range(3):
        gen = torch.Generator().manual_seed(100 + seed)
        randomize_state(ora, gen, standing=seed != 1)
        sync(ora, dev)
        dev.terrain_types.copy_(ora.terrain_types)
        t64 = float64_truth(ora, 4)
        ora.simulate(4)
        dev.simulate(4)
        torch.cuda.synchronize()
        check_derived(t64, {k: f(ora) for k, f in PHYS_QTY.items()}, {k: f(dev) for k, f in PHYS_QTY.items()})


@pytest.mark.parametrize("seed", [10, 11])
def test_post_physics_matches_oracle_philox(envs_flat, seed):
    ora, dev = envs_flat
    gen = torch.Generator().manual_seed(seed)
    randomize_state(ora, gen)
    ora._contact_forces_full[:] = (torch.rand(ora._contact_forces_full.shape, generator=gen) - 0.3) * 4
    sync(ora, dev)
    ora.common_step_counter = dev.common_step_counter = 750  # push happens at 751
    ora.post_physics_step()
    dev.post_physics_step()
    torch.cuda.synchronize()
    for name in ["obs_buf", "rew_buf", "commands", "feet_air_time", "root_states", "dof_state", "last_actions",
                 "last_dof_vel", "last_root_vel", "base_lin_vel", "base_ang_vel", "projected_gravity",
                 "_episode_sums_buf", "_extras_buf"]:
        ok, e = close(getattr(dev, name), getattr(ora, name), 1e-4, 1e-5)
        assert ok, f"{name} max err {e}"
    for name in ["reset_buf", "time_out_buf", "_episode_length_buf", "_extras_time_outs"]:
        assert torch.equal(getattr(dev, name).cpu(), getattr(ora, name)), name
    assert ora.reset_buf.any(), "test state should trigger resets"


def test_full_step_matches_oracle(envs_flat):
    ora, dev = envs_flat
    gen = torch.Generator().manual_seed(42)
    for it in range(3):
        randomize_state(ora, gen)
        sync(ora, dev)
        ora.common_step_counter = dev.common_step_counter = 10 * it
        a = (torch.rand(64, 12, generator=gen) - 0.5) * 4
        ora.step(a)
        dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf)
        ok, e = close(dev.obs_buf, ora.obs_buf, 5e-3, 5e-3)
        assert ok, f"obs max err {e}"
        ok, e = close(dev.rew_buf, ora.rew_buf, 1e-4, 1e-3)
        assert ok, f"rew max err {e}"


def test_actuator_mlp_matches_torch_and_oracle(gpu):
    from legged_gym_amd.envs.go1.go1 import pack_uninet_weights
    from legged_gym_amd.sim import lib as lgxlib
    from legged_gym_amd.sim.model import load_actuator_net
    import os
    import legged_gym_amd
    net = load_actuator_net(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources/actuator_nets/go1_net.npz"))
    rows = 4 * 256 * 4 + 7  # ragged tail
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(rows, 30, generator=gen)
    # plain torch fp32 reference of the same op (UniNet core + dVel scaling, go1.py:100-105)
    h = x
    for k in range(4):
        h = h @ torch.tensor(net[f"w{k}"]).T + torch.tensor(net[f"b{k}"])
        if k < 3:
            h = torch.tanh(h)
    ref = h * torch.tensor(net["vel_std"])
    lib = lgxlib.load()
    w = torch.tensor(pack_uninet_weights(net), device=gpu)
    scale = torch.tensor(net["vel_std"], device=gpu)
    xd = x.to(gpu)
    out = torch.empty(rows, 3, device=gpu)
    lgxlib.check(lib.lgx_actuator_mlp(C.c_void_p(xd.data_ptr()), C.c_void_p(out.data_ptr()), rows,
                                      C.c_void_p(w.data_ptr()), C.c_void_p(scale.data_ptr()), None), "mlp")
    torch.cuda.synchronize()
    ok, e = close(out, ref, 1e-4, 1e-4)
    assert ok, f"actuator mlp vs torch max err {e}"
    ol = load_oracle()
    oout = torch.empty(rows, 3)
    wt = uninet_torch_layout(w)
    scale_h = scale.cpu()
    ol.lgxo_actuator_mlp(C.c_void_p(x.data_ptr()), C.c_void_p(oout.data_ptr()), rows, C.c_void_p(wt.data_ptr()),
                         C.c_void_p(scale_h.data_ptr()))
    ok, e = close(out, oout, 1e-4, 1e-4)
    assert ok, f"actuator mlp vs oracle max err {e}"


@pytest.mark.parametrize("dims", [(48, 512, 256, 128, 12), (235, 512, 256, 128, 1), (7, 33, 5)])
def test_mlp_forward_matches_torch(gpu, dims):
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    gen = torch.Generator().manual_seed(sum(dims))
    rows = 1000
    x = torch.randn(rows, dims[0], generator=gen)
    ws = [torch.randn(dims[i + 1], dims[i], generator=gen) / dims[i] ** 0.5 for i in range(len(dims) - 1)]
    bs = [torch.randn(dims[i + 1], generator=gen) * 0.1 for i in range(len(dims) - 1)]
    h = x
    for i, (w, b) in enumerate(zip(ws, bs)):
        h = h @ w.T + b
        if i < len(ws) - 1:
            h = torch.nn.functional.elu(h)
    wts = [w.T.contiguous().to(gpu) for w in ws]
    bds = [b.to(gpu) for b in bs]
    nl = len(ws)
    dims_c = (C.c_int32 * (nl + 1))(*dims)
    wp = (C.c_void_p * nl)(*[t.data_ptr() for t in wts])
    bp = (C.c_void_p * nl)(*[t.data_ptr() for t in bds])
    xd = x.to(gpu)
    y = torch.empty(rows, dims[-1], device=gpu)
    lgxlib.check(lib.lgx_mlp_forward(C.c_void_p(xd.data_ptr()), C.c_void_p(y.data_ptr()), rows, nl, dims_c, wp, bp, 1,
                                     None), "mlp_forward")
    torch.cuda.synchronize()
    ok, e = close(y, h, 1e-4, 1e-4)
    assert ok, f"mlp forward max err {e}"


@pytest.mark.parametrize("dims,act,rows", [((235, 512, 256, 128, 12), 1, 4096), ((235, 512, 256, 128, 1), 1, 37),
                                           ((48, 512, 256, 128, 12), 1, 1000), ((7, 33, 5), 1, 1000),
                                           ((30, 128, 128, 128, 3), 2, 777)])
def test_mlp_x3_forward_matches_torch(gpu, dims, act, rows):
    """lgx_mlp_x3_forward (split-bf16 products, weights from lgx_mlp_x3_split) against a float64
    torch forward: f32-level agreement, ragged row tiles, widths off the 32 / 64 paddings."""
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    gen = torch.Generator().manual_seed(sum(dims) + rows)
    x = torch.randn(rows, dims[0], generator=gen)
    ws = [torch.randn(dims[i + 1], dims[i], generator=gen) / dims[i] ** 0.5 for i in range(len(dims) - 1)]
    bs = [torch.randn(dims[i + 1], generator=gen) * 0.1 for i in range(len(dims) - 1)]
    h = x.double()
    for i, (w, b) in enumerate(zip(ws, bs)):
        h = h @ w.double().T + b.double()
        if i < len(ws) - 1:
            h = torch.nn.functional.elu(h) if act == 1 else torch.tanh(h)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    wls = []
    for w in ws:
        wd = w.to(gpu)
        wl = torch.empty(int(lib.lgx_mlp_x3_weight_elems(w.shape[0], w.shape[1])), dtype=torch.int16, device=gpu)
        lgxlib.check(lib.lgx_mlp_x3_split(C.c_void_p(wd.data_ptr()), w.shape[0], w.shape[1], C.c_void_p(wl.data_ptr()),
                                          stream), "split")
        wls.append((wd, wl))
    bds = [b.to(gpu) for b in bs]
    xd = x.to(gpu)
    y = torch.full((rows, dims[-1]), float("nan"), device=gpu)
    d = (abi.LgxMlpX3Desc * 1)()
    d[0].x, d[0].y, d[0].rows, d[0].nl, d[0].act = xd.data_ptr(), y.data_ptr(), rows, len(ws), act
    for i, v in enumerate(dims):
        d[0].dims[i] = v
    for i in range(len(ws)):
        d[0].weights[i], d[0].biases[i] = wls[i][1].data_ptr(), bds[i].data_ptr()
    assert lib.lgx_mlp_x3_lds_bytes(d, 1) > 0
    lgxlib.check(lib.lgx_mlp_x3_forward(d, 1, stream), "mlp_x3_forward")
    torch.cuda.synchronize()
    err = (y.cpu().double() - h).abs().max().item()
    assert err <= 2e-5 * max(1.0, h.abs().max().item()), f"mlp x3 max err {err:.3e}"


def test_mlp_x3_falls_back_when_lds_is_short(gpu):
    """Three 512-wide hidden layers: 32 rows of two 512-wide limb images exceed the LDS, so the
    rollout forward runs on the f32 MFMA kernel (lgx_mlp_forward_batch) and still matches torch."""
    from legged_gym_amd.rl.actor_critic import ActorCritic
    torch.manual_seed(1)
    ac = ActorCritic(48, 48, 12, [512, 512, 512], [512, 512, 512]).to(gpu)
    obs = torch.randn(300, 48, device=gpu)
    with torch.inference_mode():
        mean, value = ac.rollout_forward(obs, obs)
        ref_mean, ref_v = ac.actor(obs), ac.critic(obs)
    assert ac._fused_actor.last_x3 is False and ac._fused_critic.last_x3 is False
    ok, e = close(mean, ref_mean, 2e-4, 2e-4)
    assert ok, f"actor mean max err {e}"
    ok, e = close(value, ref_v, 2e-4, 2e-4)
    assert ok, f"critic value max err {e}"


def test_mlp_x3_single_network_after_pair_fallback(gpu):
    """A pair that does not fit the LDS together runs f32 for that launch only: each network's own
    launch (act_inference) still takes the split-bf16 kernel when it fits alone, and a parameter
    update refreshes whichever weight image the next launch uses."""
    from legged_gym_amd.rl.actor_critic import ActorCritic, _x3_fits
    torch.manual_seed(2)
    # the actor's 32-row limb images fit the LDS alone, the critic's (512-512-256) do not
    ac = ActorCritic(235, 235, 12, [512, 256, 128], [512, 512, 256]).to(gpu)
    assert not _x3_fits([ac._fused_actor, ac._fused_critic]) and _x3_fits([ac._fused_actor])
    obs = torch.randn(300, 235, device=gpu)
    with torch.inference_mode():
        ac.rollout_forward(obs, obs)
        assert ac._fused_actor.last_x3 is False
        m1 = ac.act_inference(obs)
        assert ac._fused_actor.last_x3 is True
        ok, e = close(m1, ac.actor(obs), 2e-4, 2e-4)
        assert ok, f"actor mean max err {e}"
    with torch.no_grad():
        for p in ac.actor.parameters():
            p.add_(0.01)
    with torch.inference_mode():
        mean, _ = ac.rollout_forward(obs, obs)
        ok, e = close(mean, ac.actor(obs), 2e-4, 2e-4)
        assert ok, f"actor mean after update max err {e}"
        ok, e = close(ac.act_inference(obs), ac.actor(obs), 2e-4, 2e-4)
        assert ok, f"actor mean (split-bf16) after update max err {e}"


def test_lstm_matches_oracle(gpu):
    import os
    import legged_gym_amd
    from legged_gym_amd.envs.anymal_c.anymal import pack_lstm_weights
    from legged_gym_amd.sim import lib as lgxlib
    from legged_gym_amd.sim.model import load_actuator_net
    net = load_actuator_net(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources/actuator_nets/anydrive_v3_lstm.npz"))
    w = torch.tensor(pack_lstm_weights(net))
    m = 777
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(m, 2, generator=gen) * 0.3
    h = torch.randn(2, m, 8, generator=gen) * 0.2
    c = torch.randn(2, m, 8, generator=gen) * 0.2
    # torch fp32 reference: nn.LSTM with the same weights (anymal.py:65-77)
    lstm = torch.nn.LSTM(2, 8, 2)
    with torch.no_grad():
        for L in range(2):
            getattr(lstm, f"weight_ih_l{L}").copy_(torch.tensor(net[f"w_ih_l{L}"]))
            getattr(lstm, f"weight_hh_l{L}").copy_(torch.tensor(net[f"w_hh_l{L}"]))
            getattr(lstm, f"bias_ih_l{L}").copy_(torch.tensor(net[f"b_ih_l{L}"]))
            getattr(lstm, f"bias_hh_l{L}").copy_(torch.tensor(net[f"b_hh_l{L}"]))
        y, (h2, c2) = lstm((x * torch.tensor(net["in_scale"])).unsqueeze(0), (h, c))
        ref = (y[0] @ torch.tensor(net["w_lin"]).T + torch.tensor(net["b_lin"]))[:, 0] * float(net["out_scale"][0])
    lib = lgxlib.load()
    xd, hd, cd, wd = x.to(gpu), h.clone().to(gpu), c.clone().to(gpu), w.to(gpu)
    tau = torch.empty(m, device=gpu)
    lgxlib.check(lib.lgx_actuator_lstm(C.c_void_p(xd.data_ptr()), C.c_void_p(hd.data_ptr()), C.c_void_p(cd.data_ptr()),
                                       C.c_void_p(tau.data_ptr()), m, C.c_void_p(wd.data_ptr()), None), "lstm")
    torch.cuda.synchronize()
    for a, b, name in ((tau, ref, "tau"), (hd, h2, "h"), (cd, c2, "c")):
        ok, e = close(a, b, 1e-5, 1e-4)
        assert ok, f"lstm {name} max err {e}"


@pytest.mark.parametrize("act_mode", ["2", "1", "0"])
def test_rough_terrain_step_matches_oracle(gpu, monkeypatch, act_mode):
    """act_mode (LGX_ACT_OVERLAP, read at lgx_sim_create): the actuator net inside the post-physics
    launch (2, the default), on an auxiliary stream (1) or serially on the step's stream (0)."""
    monkeypatch.setenv("LGX_ACT_OVERLAP", act_mode)
    ora = make_env("go1_rough", num_envs=64, device="cpu", backend="oracle")
    dev = make_env("go1_rough", num_envs=64, device="cuda:0", backend="lgx")
    assert torch.equal(ora.height_samples, dev.height_samples.cpu()), "same seed -> same heightfield"
    gen = torch.Generator().manual_seed(7)
    randomize_state(ora, gen)
    sync(ora, dev)
    dev.terrain_types.copy_(ora.terrain_types)
    ora.common_step_counter = dev.common_step_counter = 3
    a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
    ora.step(a)
    dev.step(a.cuda())
    torch.cuda.synchronize()
    assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf)
    ok, e = close(dev.measured_heights, ora.measured_heights, 1e-6)
    assert ok, f"heights max err {e}"
    ok, e = close(dev.obs_buf, ora.obs_buf, 5e-3, 5e-3)
    assert ok, f"obs max err {e}"
    ok, e = close(dev.actuator_dvel, ora.actuator_dvel, 1e-3, 1e-3)
    assert ok, f"dVel max err {e}"
    for name in ["rew_buf", "_episode_sums_buf", "_extras_buf"]:
        ok, e = close(getattr(dev, name), getattr(ora, name), 1e-4, 1e-3)
        assert ok, f"{name} max err {e}"
    assert torch.equal(dev._extras_time_outs.cpu(), ora._extras_time_outs)


@pytest.mark.parametrize("bad", ["3", "-1", "2x"])
def test_unknown_act_overlap_is_refused(gpu, monkeypatch, bad):
    """LGX_ACT_OVERLAP outside {0, 1, 2} (e.g. the removed split-bf16 actuator body, 3) is refused
    by lgx_sim_create instead of silently running another mode."""
    from legged_gym_amd.sim.lib import LgxError
    monkeypatch.setenv("LGX_ACT_OVERLAP", bad)
    with pytest.raises(LgxError, match="LGX_ACT_OVERLAP"):
        make_env("go1_rough", num_envs=64, device="cuda:0", backend="lgx")


def test_mlp_forward_batch_actor_critic(gpu):
    """act_and_evaluate (one batched launch) == torch autograd modules."""
    from legged_gym_amd.rl.actor_critic import ActorCritic
    torch.manual_seed(0)
    ac = ActorCritic(235, 235, 12, [512, 256, 128], [512, 256, 128]).to(gpu)
    obs = torch.randn(4096 + 5, 235, device=gpu)
    with torch.inference_mode():
        _, v = ac.act_and_evaluate(obs, obs)
        mean = ac.action_mean
        ref_mean = ac.actor(obs)
        ref_v = ac.critic(obs)
    ok, e = close(mean, ref_mean, 2e-4, 2e-4)
    assert ok, f"actor mean max err {e}"
    ok, e = close(v, ref_v, 2e-4, 2e-4)
    assert ok, f"critic value max err {e}"
    assert ac._fused_actor.last_x3 and ac._fused_critic.last_x3   # the split-bf16 kernel ran


@pytest.mark.parametrize("N", [1000, 4096, 3])
def test_gae_kernel_matches_torch_loop(gpu, N):
    """lgx_gae_norm (GAE + rsl_rl's advantage normalisation, unbiased std) vs the torch loop."""
    from legged_gym_amd.rl.storage import RolloutStorage
    T = 24
    gen = torch.Generator().manual_seed(1)
    st_c = RolloutStorage(N, T, [4], [None], [2], "cpu")
    st_c.rewards.copy_(torch.randn(T, N, 1, generator=gen))
    st_c.values.copy_(torch.randn(T, N, 1, generator=gen))
    st_c.dones.copy_((torch.rand(T, N, 1, generator=gen) < 0.1).byte())
    last = torch.randn(N, 1, generator=gen)
    st_g = RolloutStorage(N, T, [4], [None], [2], str(gpu))
    for name in ("rewards", "values", "dones"):
        getattr(st_g, name).copy_(getattr(st_c, name))
    st_c.compute_returns(last, 0.99, 0.95)
    st_g.compute_returns(last.to(gpu), 0.99, 0.95)
    ok, e = close(st_g.returns, st_c.returns, 1e-4, 1e-5)
    assert ok, f"returns max err {e}"
    ok, e = close(st_g.advantages, st_c.advantages, 1e-4, 1e-4)
    assert ok, f"advantages max err {e}"


def test_gae_norm_large_mean_advantages(gpu):
    """Advantages with |mean| >> std (rewards ~3e3 +- 1e-2): the per-workgroup (count, mean, M2)
    summaries combined with Chan's formula keep the normalised advantages at float64 accuracy (a
    one-pass sum-of-squares variance cancels to nothing here)."""
    from legged_gym_amd.rl.storage import RolloutStorage
    T, N = 24, 4096
    gen = torch.Generator().manual_seed(2)
    st = RolloutStorage(N, T, [4], [None], [2], str(gpu))
    rew = 3e3 + 1e-2 * torch.randn(T, N, 1, generator=gen)
    st.rewards.copy_(rew)
    st.values.zero_()
    st.dones.zero_()
    last = torch.zeros(N, 1)
    st.compute_returns(last.to(gpu), 0.0, 0.95)   # gamma 0: advantage = reward - value
    adv = st.returns.double().cpu()            # values are zero: raw advantages = returns
    want = (adv - adv.mean()) / (adv.std() + 1e-8)
    got = st.advantages.double().cpu()
    assert (got - want).abs().max().item() <= 2e-3 * want.abs().max().item()
    assert abs(got.std().item() - 1.0) < 1e-3


@pytest.mark.parametrize("mean", [0.0, 3e3])
def test_dp_advantage_statistics_match_gae_norm(gpu, mean):
    """The data-parallel normalisation (lgx_gae_parts -> gathered summaries -> lgx_adv_norm) at
    world 1 is bitwise lgx_gae_norm's, and over two shards it equals the one-process statistics of
    the whole batch (the DP path keeps Chan's float64 moments, also when |mean| >> std)."""
    from legged_gym_amd.rl.storage import RolloutStorage
    T, N = 24, 4096
    gen = torch.Generator().manual_seed(3)
    rew = mean + torch.randn(T, N, 1, generator=gen) * (1e-2 if mean else 1.0)
    val = torch.randn(T, N, 1, generator=gen) * (1e-3 if mean else 1.0)
    dones = (torch.rand(T, N, 1, generator=gen) < 0.05).byte()
    last = torch.randn(N, 1, generator=gen)

    def mk(sl):
        st = RolloutStorage(sl.stop - sl.start, T, [4], [None], [2], str(gpu))
        st.rewards.copy_(rew[:, sl]), st.values.copy_(val[:, sl]), st.dones.copy_(dones[:, sl])
        return st
    full = slice(0, N)
    one, dp1 = mk(full), mk(full)
    one.compute_returns(last.to(gpu), 0.99, 0.95)
    dp1.compute_returns(last.to(gpu), 0.99, 0.95, reduce_stats=lambda p: p)
    assert torch.equal(one.advantages, dp1.advantages) and torch.equal(one.returns, dp1.returns)
    # two "ranks" of N/2 envs: gather both ranks' GAE summaries in rank order, normalise each shard
    from legged_gym_amd.rl import fused
    shards = [mk(slice(0, N // 2)), mk(slice(N // 2, N))]
    parts = [fused.gae_parts(s.rewards, s.values, s.dones, last[sl].to(gpu).contiguous(), s.returns, s.advantages,
                             0.99, 0.95) for s, sl in zip(shards, (slice(0, N // 2), slice(N // 2, N)))]
    allp = torch.cat(parts)
    for s in shards:
        fused.adv_norm(s.advantages, allp)
    got = torch.cat([s.advantages for s in shards], dim=1)
    assert (got - one.advantages).abs().max().item() <= 1e-5 * max(1.0, one.advantages.abs().max().item())


def test_splitk_linear_gradients_match_torch(gpu):
    from legged_gym_amd.rl.actor_critic import LgxLinear
    torch.manual_seed(0)
    lin = LgxLinear(235, 512).to(gpu)
    ref = torch.nn.Linear(235, 512).to(gpu)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(24576, 235, device=gpu, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    g = torch.randn(24576, 512, device=gpu)
    (lin(x) * g).sum().backward()
    (ref(x2) * g).sum().backward()
    for a, b in ((lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad), (x.grad, x2.grad)):
        ok, e = close(a, b, 1e-2, 1e-4)
        assert ok, f"split-K grad max err {e}"


@pytest.mark.parametrize("ctrl", ["P", "V", "T"])
def test_explicit_torque_control_matches_oracle(gpu, ctrl):
    """_compute_torques (legged_robot.py:370-392) instead of the position drive: one env step."""
    def ov(c):
        c.control.explicit_torques = True
        c.control.control_type = ctrl
        if ctrl == "V":
            # Go1's gains make explicit velocity control unstable at sim dt (Kp dt / I_calf ~ 100,
            # saturated bang-bang): compare on gains the explicit integrator resolves
            c.control.stiffness = {k: 0.1 for k in c.control.stiffness}
            c.control.damping = {k: 1e-5 for k in c.control.damping}
    ora = make_env("go1_flat_bench", num_envs=64, device="cpu", backend="oracle", overrides=ov)
    dev = make_env("go1_flat_bench", num_envs=64, device="cuda:0", backend="lgx", overrides=ov)
    gen = torch.Generator().manual_seed(21)
    randomize_state(ora, gen)
    sync(ora, dev)
    a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
    ora.step(a)
    dev.step(a.cuda())
    torch.cuda.synchronize()
    ok, e = close(dev.torques, ora.torques, 1e-3, 1e-3)
    assert ok, f"torques max err {e}"
    assert (dev.torques.abs() <= dev.torque_limits + 1e-4).all()
    ok, e = close(dev.dof_state, ora.dof_state, 5e-3, 2e-3)
    assert ok, f"dof max err {e}"
    ok, e = close(dev.obs_buf, ora.obs_buf, 5e-3, 5e-3)
    assert ok, f"obs max err {e}"


@pytest.mark.parametrize("task", ["a1", "a1_src", "aliengo", "anymal_b"])
def test_other_robots_step_matches_oracle(gpu, task):
    """The remaining registered quadrupeds (model JSONs from their URDFs): one full env step
    from a randomised state, HIP path vs oracle."""
    ora = make_env(task, num_envs=64, device="cpu", backend="oracle")
    dev = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    gen = torch.Generator().manual_seed(21)
    randomize_state(ora, gen)
    sync(ora, dev)
    dev.terrain_types.copy_(ora.terrain_types)
    ora.common_step_counter = dev.common_step_counter = 5
    a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
    ora.step(a)
    dev.step(a.cuda())
    torch.cuda.synchronize()
    assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf)
    keep = ~ora.reset_buf
    ok, e = close(dev.root_states.cpu()[keep], ora.root_states[keep], 2e-3, 2e-3)
    assert ok, f"root max err {e}"
    ok, e = close(dev.obs_buf.cpu()[keep], ora.obs_buf[keep], 5e-3, 5e-3)
    assert ok, f"obs max err {e}"
    ok, e = close(dev.rew_buf.cpu()[keep], ora.rew_buf[keep], 1e-4, 1e-3)
    assert ok, f"rew max err {e}"


@pytest.mark.parametrize("pp", ["4", "2", "1"])
def test_anymal_c_rough_dr_step_matches_oracle(gpu, monkeypatch, pp):
    """BASELINE C5 (anymal_c_rough_config.py:33-94): ANYmal-C on the curriculum trimesh with the
    full domain randomisation - friction buckets U[0.5, 1.25] (legged_robot.py:259-282), base mass
    +U[-5, 5] kg (anymal_c_rough_config.py:80-81, legged_robot.py:312-335) and the push at step
    751 (legged_robot.py:436-441) - two env steps, HIP path vs oracle.  pp = LGX_PHYS_PP: every
    lane split of lgx_physics_kernel (4 = the default at every size; 2 and 1 as A/B variants)."""
    monkeypatch.setenv("LGX_PHYS_PP", pp)
    ora = make_env("anymal_c_rough", num_envs=64, device="cpu", backend="oracle")
    dev = make_env("anymal_c_rough", num_envs=64, device="cuda:0", backend="lgx")
    assert torch.equal(ora.height_samples, dev.height_samples.cpu()), "same seed -> same heightfield"
    # the randomisation is live: per-env friction from the 64 buckets, base masses spread over +-5 kg
    assert ora.friction_coeffs.unique().numel() > 8 and ora.friction_coeffs.min() >= 0.5 and ora.friction_coeffs.max() <= 1.25
    base = ora.body_masses[:, 0] - ora.asset.data["report_bodies"][0]["mass"]
    assert base.min() >= -5 and base.max() <= 5 and base.std() > 1.5
    assert ora.cfg.domain_rand.push_robots and int(ora.cfg.domain_rand.push_interval) == 751
    gen = torch.Generator().manual_seed(77)
    randomize_state(ora, gen)
    ora._episode_length_buf[:4] = int(ora.max_episode_length)     # envs 0-3 time out in the first step
    sync(ora, dev)
    dev.terrain_types.copy_(ora.terrain_types)
    ora.common_step_counter = dev.common_step_counter = 749       # the second step is the push step
    for it in range(2):
        a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
        ora.step(a)
        dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf), it
        assert torch.equal(dev._episode_length_buf.cpu(), ora._episode_length_buf), it
        keep = ~ora.reset_buf
        ok, e = close(dev.root_states.cpu()[keep], ora.root_states[keep], 2e-3, 2e-3)
        assert ok, f"step {it}: root max err {e}"
        ok, e = close(dev.dof_state.view(64, 12, 2).cpu()[keep], ora.dof_state.view(64, 12, 2)[keep], 5e-3, 2e-3)
        assert ok, f"step {it}: dof max err {e}"
        ok, e = close(dev.measured_heights, ora.measured_heights, 1e-6)
        assert ok, f"step {it}: heights max err {e}"
        ok, e = close(dev.obs_buf.cpu()[keep], ora.obs_buf[keep], 5e-3, 5e-3)
        assert ok, f"step {it}: obs max err {e}"
        ok, e = close(dev.rew_buf.cpu()[keep], ora.rew_buf[keep], 1e-4, 1e-3)
        assert ok, f"step {it}: rew max err {e}"
        # reset envs: the reset state itself (Philox draws keyed by env index)
        assert it == 1 or (~keep).sum() >= 4
        if (~keep).any():
            ok, e = close(dev.root_states.cpu()[~keep], ora.root_states[~keep], 1e-4, 1e-5)
            assert ok, f"step {it}: reset root max err {e}"
        if it == 0:   # the push step starts from identical states (contacts amplify rounding)
            sync(ora, dev)
    assert torch.equal(dev.terrain_levels.cpu(), ora.terrain_levels)


@pytest.mark.parametrize("pp", ["4", "2", "1"])
def test_anymal_sea_torque_step_matches_oracle(gpu, monkeypatch, pp):
    """ANYmal-C with the SEA actuator network as the torque source (LGX_CTRL_SEA: anymal.py:71-78 via
    cfg.control.explicit_torques; the LSTM advanced in the physics launch once per substep, its
    joints dealt over the PP lanes of each leg): three env steps from a randomised state with
    non-zero LSTM state, envs 0-3 timing out in the first step (their LSTM state restarts from zero
    in the second, anymal.py:56-60), HIP path vs oracle; every lane split of the kernel."""
    monkeypatch.setenv("LGX_PHYS_PP", pp)

    def ov(c):
        c.control.explicit_torques = True
    ora = make_env("anymal_c_rough", num_envs=64, device="cpu", backend="oracle", overrides=ov)
    dev = make_env("anymal_c_rough", num_envs=64, device="cuda:0", backend="lgx", overrides=ov)
    from legged_gym_amd.sim import abi
    assert dev._lgx_params.control_type == abi.CTRL["SEA"]
    gen = torch.Generator().manual_seed(31)
    randomize_state(ora, gen)
    ora._episode_length_buf[:4] = int(ora.max_episode_length)
    ora.sea_hidden_state.copy_(torch.randn(2, 64 * 12, 8, generator=gen) * 0.3)
    ora.sea_cell_state.copy_(torch.randn(2, 64 * 12, 8, generator=gen) * 0.3)
    sync(ora, dev)
    dev.terrain_types.copy_(ora.terrain_types)
    ora.common_step_counter = dev.common_step_counter = 3
    for it in range(3):
        dev.sea_hidden_state.copy_(ora.sea_hidden_state)
        dev.sea_cell_state.copy_(ora.sea_cell_state)
        a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
        ora.step(a)
        dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf), it
        if it == 0:
            assert ora.reset_buf[:4].all()
        if it == 0:   # reset_idx zeroed the LSTM state of the envs that reset (anymal.py:56-60)
            assert (dev.sea_hidden_state.view(2, 64, 12, 8)[:, :4] == 0).all()
            assert (dev.sea_cell_state.view(2, 64, 12, 8)[:, :4] == 0).all()
            assert (dev.sea_hidden_state.view(2, 64, 12, 8)[:, 4:] != 0).any()
        if it == 1:   # the envs reset by step 0 restarted their LSTM state from zero
            assert (dev._episode_length_buf[:4] == 1).all()
        # LSTM state after 4 substeps: f32 with fma contraction and v_exp-based sigmoid / tanh in
        # the kernel vs libm expf / tanhf without contraction in the oracle, through the recurrence
        ok, e = close(dev.sea_hidden_state, ora.sea_hidden_state, 2e-4, 1e-4)
        assert ok, f"step {it}: sea h max err {e}"
        ok, e = close(dev.sea_cell_state, ora.sea_cell_state, 2e-4, 1e-4)
        assert ok, f"step {it}: sea c max err {e}"
        ok, e = close(dev.torques, ora.torques, 2e-3, 1e-3)
        assert ok, f"step {it}: torques max err {e}"
        assert (dev.torques.abs() <= dev.torque_limits + 1e-4).all()
        keep = ~ora.reset_buf
        ok, e = close(dev.dof_state.view(64, 12, 2).cpu()[keep], ora.dof_state.view(64, 12, 2)[keep], 5e-3, 2e-3)
        assert ok, f"step {it}: dof max err {e}"
        ok, e = close(dev.root_states.cpu()[keep], ora.root_states[keep], 2e-3, 2e-3)
        assert ok, f"step {it}: root max err {e}"
        ok, e = close(dev.obs_buf.cpu()[keep], ora.obs_buf[keep], 5e-3, 5e-3)
        assert ok, f"step {it}: obs max err {e}"
        sync(ora, dev)   # next step from identical states


def test_direct_actions_and_extras_snapshots(gpu):
    """lgx_step_from (policy tensor read in place) == copy-then-lgx_step, the caller's tensor is not
    clipped in place, and every step publishes its own extras snapshot (kernel-written) that
    stays valid after later steps, as the reference's fresh tensors do."""
    a_env = make_env("go1_rough", num_envs=64, device="cuda:0", backend="lgx")
    b_env = make_env("go1_rough", num_envs=64, device="cuda:0", backend="lgx")
    a_env.reset()
    b_env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    kept, expect = [], []
    for _ in range(30):
        act = torch.randn(64, 12, device="cuda:0", generator=gen) * 150.0   # beyond clip_actions
        raw = act.clone()
        assert a_env._direct_actions(act) and not b_env._direct_actions(act.t().contiguous().t())
        oa, _, ra, da, ia = a_env.step(act)
        ob, _, rb, db, ib = b_env.step(act.t().contiguous().t())
        assert torch.equal(act, raw)
        assert torch.equal(a_env.actions, b_env.actions) and a_env.actions.abs().max() <= 100.0
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
        kept.append(ia["episode"])
        expect.append(a_env._extras_buf.clone())
    for ep, ref in zip(kept, expect):
        for key, row in a_env._extras_rows:
            assert torch.equal(ep[key], ref[row]), key


def _cassie_state(env, gen):
    """randomize_state at the biped's standing height (pelvis ~0.9 m) with its feet near the ground."""
    randomize_state(env, gen)
    N = env.num_envs
    env.root_states[:, 2] = env.env_origins[:, 2] + 0.80 + 0.15 * torch.rand(N, generator=gen)


@pytest.mark.parametrize("seed", [0, 1])
def test_cassie_dense_physics_matches_float64(gpu, seed):
    """Cassie (2 legs x 6 joints: lgx_physics_dense_kernel) on its rough terrain: 4 substeps from
    randomised states, HIP vs the float64 oracle with the derived tolerance (check_derived)."""
    ora = make_env("cassie", num_envs=64, device="cpu", backend="oracle")
    dev = make_env("cassie", num_envs=64, device="cuda:0", backend="lgx")
    assert dev._lgx_model.leg_dof == 6
    gen = torch.Generator().manual_seed(200 + seed)
    _cassie_state(ora, gen)
    sync(ora, dev)
    dev.terrain_types.copy_(ora.terrain_types)
    t64 = float64_truth(ora, 4)
    ora.simulate(4)
    dev.simulate(4)
    torch.cuda.synchronize()
    errs = check_derived(t64, {k: f(ora) for k, f in PHYS_QTY.items()}, {k: f(dev) for k, f in PHYS_QTY.items()})
    assert ora.contact_forces[:, ora.feet_indices].abs().sum() > 0, "the test states should touch the ground"
    assert errs["dof_vel"][0] < 0.05, errs


def test_cassie_full_step_matches_oracle(gpu):
    """lgx_step on the biped (dense physics + the env-logic kernel with no_fly, 2 feet, the 11 x 11
    scan and pelvis termination) vs the oracle, 3 steps from randomised states."""
    ora = make_env("cassie", num_envs=64, device="cpu", backend="oracle")
    dev = make_env("cassie", num_envs=64, device="cuda:0", backend="lgx")
    gen = torch.Generator().manual_seed(42)
    for it in range(3):
        _cassie_state(ora, gen)
        sync(ora, dev)
        dev.terrain_types.copy_(ora.terrain_types)
        ora.common_step_counter = dev.common_step_counter = 10 * it
        a = (torch.rand(64, 12, generator=gen) - 0.5) * 2
        ora.step(a)
        dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(dev.reset_buf.cpu(), ora.reset_buf), it
        keep = ~ora.reset_buf
        ok, e = close(dev.obs_buf.cpu()[keep], ora.obs_buf[keep], 5e-3, 5e-3)
        assert ok, f"obs max err {e}"
        ok, e = close(dev.rew_buf.cpu()[keep], ora.rew_buf[keep], 1e-4, 1e-3)
        assert ok, f"rew max err {e}"
        ok, e = close(dev.feet_air_time, ora.feet_air_time, 1e-5)
        assert ok, f"feet air time max err {e}"


@pytest.mark.parametrize("task", ["go1_flat_bench", "anymal_c_rough"])
def test_dense_kernel_on_quadrupeds_matches_float64(gpu, monkeypatch, task):
    """The dense joint-space kernel is a second, independent GPU formulation of the same physics
    (LGX_PHYS_DENSE=1 selects it for the 4 x 3 quadrupeds): HIP vs the float64 oracle with the derived
    tolerance, and vs the arrowhead kernel's result from the same state."""
    ora = make_env(task, num_envs=64, device="cpu", backend="oracle")
    arrow = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    monkeypatch.setenv("LGX_PHYS_DENSE", "1")
    dense = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    gen = torch.Generator().manual_seed(7)
    randomize_state(ora, gen)
    for dev in (arrow, dense):
        sync(ora, dev)
        dev.terrain_types.copy_(ora.terrain_types)
    t64 = float64_truth(ora, 4)
    ora.simulate(4)
    arrow.simulate(4)
    dense.simulate(4)
    torch.cuda.synchronize()
    ov = {k: f(ora) for k, f in PHYS_QTY.items()}
    check_derived(t64, ov, {k: f(dense) for k, f in PHYS_QTY.items()})
    check_derived(t64, ov, {k: f(arrow) for k, f in PHYS_QTY.items()})


def test_sim_buffer_reports_the_bound_tensors(gpu):
    """lgx_sim_buffer: every id names the tensor the env bound at lgx_sim_create
    (obs: the one rebound by the latest step), with its shape and dtype; an unknown id fails."""
    env = make_env("go1_rough", num_envs=64, device="cuda:0", backend="lgx")
    env.step(torch.zeros(env.num_envs, env.num_actions, device=env.device))
    torch.cuda.synchronize()
    be = env._backend
    bound = {"root_states": env.root_states, "dof_state": env.dof_state, "dof_targets": env.target_poses,
             "torques": env.torques, "contact_forces": env._contact_forces_full, "actions": env.actions,
             "last_actions": env.last_actions, "last_dof_vel": env.last_dof_vel, "last_root_vel": env.last_root_vel,
             "commands": env.commands, "base_lin_vel": env.base_lin_vel, "base_ang_vel": env.base_ang_vel,
             "projected_gravity": env.projected_gravity, "feet_air_time": env._feet_air_time_full,
             "obs": env.obs_buf, "rew": env.rew_buf, "reset": env.reset_buf, "time_out": env.time_out_buf,
             "episode_length": env._episode_length_buf, "episode_sums": env._episode_sums_buf,
             "measured_heights": env.measured_heights, "env_origins": env.env_origins,
             "terrain_levels": env.terrain_levels, "terrain_types": env.terrain_types, "extras": env._extras_buf}
    assert set(bound) == set(be.BUFFER_IDS)
    for name in be.BUFFER_IDS:
        ptr, shape, dtype = be.buffer(name)
        t = bound[name]
        assert ptr == t.data_ptr(), name
        assert dtype == (torch.uint8 if t.dtype == torch.bool else t.dtype), name
        assert int(np.prod(shape)) == t.numel(), (name, shape, tuple(t.shape))
        if name != "dof_state":   # (the reference's view is [N * 12, 2], gymtorch's wrap of the same memory)
            assert shape[0] == t.shape[0], name
    assert be.buffer("dof_state")[1] == (64, 12, 2)
    assert be.buffer("contact_forces")[1] == (64, 17, 3)
    assert be.buffer("obs")[1] == (64, env.num_obs)
    ptr, shape, nd, dt = C.c_void_p(), (C.c_int64 * 4)(), C.c_int32(), C.c_int32()
    assert be.lib.lgx_sim_buffer(be.handle, len(be.BUFFER_IDS), C.byref(ptr), shape, C.byref(nd), C.byref(dt)) != 0
    assert b"unknown buffer id" in be.lib.lgx_last_error()
