"""CPU: the float64 oracle's branch records and forced branches (lgxo_branch_trace /
lgxo_branch_force), which tests/test_gpu_parity.py uses to explain physics outliers by a
near-threshold flip instead of allowing them: a forced run that takes every recorded decision
reproduces the free run bitwise; flipping a decision changes only the env that owns it; and the
records carry every kind of decision with a finite margin."""
import torch

from oracle_backend import BRANCH_ALTERNATIVES, make_env, simulate64
from test_gpu_parity import PHYS_QTY, PHYS_STATE, float64_truth, randomize_state


def _env(task="go1_rough"):
    ora = make_env(task, num_envs=16, device="cpu", backend="oracle")
    randomize_state(ora, torch.Generator().manual_seed(3), standing=True)
    return ora


def test_records_cover_every_decision_kind():
    ora = _env()
    t = float64_truth(ora, 4)
    kinds = {r[2] for r in t.records}
    assert kinds == {1, 2, 3, 4}, kinds
    assert all(abs(r[5]) < float("inf") for r in t.records)
    # drives: one record per joint, env and substep
    assert sum(1 for r in t.records if r[2] == 1) == 16 * 4 * 12
    for r in t.records:
        assert r[4] in BRANCH_ALTERNATIVES[r[2]]


def test_forcing_the_recorded_decisions_reproduces_the_run():
    ora = _env()
    t = float64_truth(ora, 4)
    same = t.forced([r[:5] for r in t.records])
    for k in PHYS_QTY:
        assert torch.equal(same[k], t[k]), k


def test_a_flip_changes_only_its_env():
    ora = _env()
    t = float64_truth(ora, 4)
    r = next(r for r in t.records if r[2] == 1 and r[1] == 0)           # a drive decision at substep 0
    flipped = t.forced([(r[0], r[1], r[2], r[3], 1 - r[4])])
    e = r[0]
    changed = {k for k in PHYS_QTY if not torch.equal(flipped[k][e], t[k][e])}
    assert "dof_vel" in changed
    others = [i for i in range(16) if i != e]
    for k in PHYS_QTY:
        assert torch.equal(flipped[k][others], t[k][others]), k
    # the oracle env's own state is untouched by truth / forced runs
    s = {k: getattr(ora, k).clone() for k in PHYS_STATE}
    t.forced([(r[0], r[1], r[2], r[3], 1 - r[4])])
    for k in PHYS_STATE:
        assert torch.equal(getattr(ora, k), s[k])


def _drive_edge_state(margin):
    """go1_flat_bench, 16 envs, randomised; env 0 joint 0's PD torque placed at `margin` past the
    effort limit (saturated) in the first substep."""
    ora = make_env("go1_flat_bench", num_envs=16, device="cpu", backend="oracle")
    randomize_state(ora, torch.Generator().manual_seed(11), standing=True)
    m = ora._lgx_model
    kp, kd, eff = float(m.kp[0]), float(m.kd[0]), float(m.dof_effort[0])
    th, thd = float(ora.dof_pos[0, 0]), float(ora.dof_vel[0, 0])
    ora.target_poses[0, 0] = th + (eff * (1 + margin) + kd * thd) / kp
    return ora


def test_explain_outliers_finds_a_near_threshold_flip():
    """The explanation search end to end on CPU: a 'device' result that took the other branch of a
    drive decision 1e-4 past its threshold (a forced float64 run) is an outlier against the float64
    truth, and check_derived explains it by exactly that flip."""
    import test_gpu_parity as P
    ora = _drive_edge_state(1e-4)
    t = float64_truth(ora, 4)
    rec = [r for r in t.records if r[:4] == (0, 0, 1, 0)]
    assert len(rec) == 1 and rec[0][4] == 0 and abs(rec[0][5] - 1e-4) < 1e-6, rec
    dev = t.forced([(0, 0, 1, 0, 1)])                      # the other branch: implicit drive
    ora.simulate(4)                                        # the float32 oracle takes the truth's branch
    ora_vals = {k: f(ora) for k, f in PHYS_QTY.items()}
    n0 = len(P.BRANCH_FLIPS)
    P.check_derived(t, ora_vals, dev)
    flips = P.BRANCH_FLIPS[n0:]
    assert len(flips) == 1 and flips[0]["env"] == 0, flips
    assert flips[0]["flips"] == [("drive", "substep 0", "index 0", "-> 1")]
    assert abs(flips[0]["margins"][0] - 1e-4) < 1e-6


def test_unexplained_outlier_fails():
    """An env far from the float64 truth that no near-threshold flip explains fails check_derived."""
    import pytest
    import test_gpu_parity as P
    ora = _drive_edge_state(0.5)                           # (no decision near its threshold there)
    t = float64_truth(ora, 4)
    dev = {k: v.clone() for k, v in t.items()}
    dev["root_vel"][3] += 1e-2                             # a bug-sized error in env 3
    ora.simulate(4)
    with pytest.raises(AssertionError, match="env 3"):
        P.check_derived(t, {k: f(ora) for k, f in PHYS_QTY.items()}, dev)
