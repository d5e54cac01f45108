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
