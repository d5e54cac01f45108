"""PPO / storage / runner tests on CPU, and the data-parallel path with gloo (world_size 2).

rsl_rl is absent from the container and unpinned: parity of the PPO math is
UNPINNED against the upstream package; these tests pin it against an independent numpy
restatement of the published rsl_rl v1.0.x equations and check that N ranks x B envs equal
1 rank x N*B envs (the data-parallel contract).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from legged_gym_amd.rl.actor_critic import ActorCritic
from legged_gym_amd.rl.ppo import PPO
from legged_gym_amd.rl.storage import RolloutStorage

T, B, OBS, ACT = 6, 32, 10, 3


def gae_numpy(r, v, d, last, gamma, lam):
    Tn = r.shape[0]
    ret = np.zeros_like(r)
    adv = 0.0
    for t in reversed(range(Tn)):
        nv = last if t == Tn - 1 else v[t + 1]
        nt = 1.0 - d[t]
        delta = r[t] + nt * gamma * nv - v[t]
        adv = delta + nt * gamma * lam * adv
        ret[t] = adv + v[t]
    a = ret - v
    return ret, (a - a.mean()) / (a.std(ddof=1) + 1e-8)


def fill(storage, gen, n_envs, offset=0):
    """Deterministic transitions for envs [offset, offset + n_envs) of a global batch."""
    g = torch.Generator().manual_seed(1234)
    full = {
        "obs": torch.randn(T, 2 * B, OBS, generator=g),
        "act": torch.randn(T, 2 * B, ACT, generator=g),
        "rew": torch.randn(T, 2 * B, 1, generator=g),
        "done": (torch.rand(T, 2 * B, 1, generator=g) < 0.15).byte(),
        "val": torch.randn(T, 2 * B, 1, generator=g),
        "logp": torch.randn(T, 2 * B, 1, generator=g) - 3,
        "mu": torch.randn(T, 2 * B, ACT, generator=g) * 0.1,
        "sigma": torch.ones(T, 2 * B, ACT),
    }
    sl = slice(offset, offset + n_envs)
    storage.observations.copy_(full["obs"][:, sl])
    storage.actions.copy_(full["act"][:, sl])
    storage.rewards.copy_(full["rew"][:, sl])
    storage.dones.copy_(full["done"][:, sl])
    storage.values.copy_(full["val"][:, sl])
    storage.actions_log_prob.copy_(full["logp"][:, sl])
    storage.mu.copy_(full["mu"][:, sl])
    storage.sigma.copy_(full["sigma"][:, sl])
    storage.step = T
    return full


def make_alg(n_envs, epochs=2, mbs=1):
    torch.manual_seed(0)
    ac = ActorCritic(OBS, OBS, ACT, [16, 8], [16, 8])
    alg = PPO(ac, num_learning_epochs=epochs, num_mini_batches=mbs, learning_rate=1e-3, gamma=0.99, lam=0.95,
              schedule="adaptive", entropy_coef=0.01, device="cpu")
    alg.init_storage(n_envs, T, [OBS], [None], [ACT])
    return alg


def test_gae_matches_numpy_restatement():
    alg = make_alg(2 * B)
    full = fill(alg.storage, None, 2 * B)
    last = torch.randn(2 * B, 1, generator=torch.Generator().manual_seed(9))
    alg.storage.compute_returns(last, 0.99, 0.95)
    ret, adv = gae_numpy(full["rew"].numpy(), full["val"].numpy(), full["done"].numpy().astype(np.float32),
                         last.numpy(), 0.99, 0.95)
    np.testing.assert_allclose(alg.storage.returns.numpy(), ret, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(alg.storage.advantages.numpy(), adv, rtol=1e-4, atol=1e-5)


def test_update_runs_and_adapts_lr():
    alg = make_alg(2 * B, epochs=2, mbs=2)
    fill(alg.storage, None, 2 * B)
    alg.storage.compute_returns(torch.zeros(2 * B, 1), 0.99, 0.95)
    # old_sigma far from current sigma -> huge KL -> lr divided by 1.5 per minibatch
    alg.storage.sigma.fill_(0.1)
    p0 = [p.clone() for p in alg.actor_critic.parameters()]
    vl, sl = alg.update()
    assert np.isfinite(vl) and np.isfinite(sl)
    assert alg.learning_rate == pytest.approx(1e-3 / 1.5 ** 4)
    assert any(not torch.equal(a, b) for a, b in zip(p0, alg.actor_critic.parameters()))


@pytest.mark.parametrize("schedule,sigma,clipped_v,mbs", [("adaptive", 1.0, True, 2), ("adaptive", 0.1, True, 2),
                                                          ("fixed", 1.0, False, 3)])
def test_update_matches_numpy_oracle(schedule, sigma, clipped_v, mbs):
    """PPO.update (autograd, CPU float32) against oracle/ppo_oracle.py, the hand-differentiated
    numpy float64 restatement of rsl_rl's PPO.update (minibatch order, clipped surrogate /
    value loss, entropy, adaptive KL learning rate, clip_grad_norm_, Adam).  sigma 0.1: the
    rollout's std far from the policy's -> the learning rate falls at every minibatch."""
    from ppo_oracle_io import oracle_update, param_deviation
    alg = make_alg(2 * B, epochs=2, mbs=mbs)
    alg.schedule = schedule
    alg.use_clipped_value_loss = clipped_v
    fill(alg.storage, None, 2 * B)
    alg.storage.sigma.fill_(sigma)
    alg.storage.compute_returns(torch.randn(2 * B, 1, generator=torch.Generator().manual_seed(5)), 0.99, 0.95)
    want = oracle_update(alg, seed=21)
    torch.manual_seed(21)
    vl, sl = alg.update()
    assert alg.learning_rate == pytest.approx(want[3], rel=1e-12)
    assert vl == pytest.approx(want[4], rel=1e-5, abs=1e-7) and sl == pytest.approx(want[5], rel=1e-5, abs=1e-7)
    dmax, big, total = param_deviation(alg.actor_critic, want)
    n_steps = 2 * mbs
    assert dmax <= 2 * n_steps * 1e-3, dmax
    assert big <= max(2, 1e-3 * total), (big, total)


def test_update_matches_numpy_oracle_policy_widths():
    """The same at the go1_rough policy widths (235 -> 512 -> 256 -> 128 -> 12 / 1), 2 epochs x 4
    minibatches: at this size the value-clipping branches include in-range rows where rounding
    makes tv + (v - tv) != v (torch routes the whole gradient through the larger branch)."""
    from ppo_oracle_io import oracle_update, param_deviation
    Tn, Nn, obs_n, act_n = 4, 96, 235, 12
    torch.manual_seed(0)
    ac = ActorCritic(obs_n, obs_n, act_n, [512, 256, 128], [512, 256, 128])
    alg = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95, value_loss_coef=1.0,
              entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0, schedule="adaptive", desired_kl=0.01,
              device="cpu")
    alg.init_storage(Nn, Tn, [obs_n], [None], [act_n])
    g = torch.Generator().manual_seed(3)
    st = alg.storage
    st.observations.copy_(torch.randn(Tn, Nn, obs_n, generator=g))
    st.actions.copy_(torch.randn(Tn, Nn, act_n, generator=g))
    st.rewards.copy_(torch.randn(Tn, Nn, 1, generator=g))
    st.dones.copy_((torch.rand(Tn, Nn, 1, generator=g) < 0.1).byte())
    st.values.copy_(torch.randn(Tn, Nn, 1, generator=g))
    st.actions_log_prob.copy_(torch.randn(Tn, Nn, 1, generator=g) * 0.3 - 17)
    st.mu.copy_(torch.randn(Tn, Nn, act_n, generator=g) * 0.1)
    st.sigma.copy_(torch.rand(Tn, Nn, act_n, generator=g) * 0.5 + 0.75)
    st.step = Tn
    st.compute_returns(torch.randn(Nn, 1, generator=g), 0.99, 0.95)
    want = oracle_update(alg, seed=13)
    torch.manual_seed(13)
    vl, sl = alg.update()
    assert alg.learning_rate == pytest.approx(want[3], rel=1e-12)
    assert vl == pytest.approx(want[4], rel=1e-5) and sl == pytest.approx(want[5], rel=1e-5)
    dmax, big, total = param_deviation(alg.actor_critic, want)
    assert dmax <= 2 * 8 * 1e-3, dmax
    assert big <= 1e-3 * total, (big, total)


def test_minibatch_gradient_matches_numpy_oracle():
    """d loss / d parameters of one minibatch (autograd, CPU float32) against the oracle's
    hand-derived float64 gradient: |d| <= 1e-5 + 1e-4 |g|."""
    from ppo_oracle_io import oracle_minibatch_grads, grad_deviation
    alg = make_alg(2 * B, epochs=1, mbs=2)
    fill(alg.storage, None, 2 * B)
    alg.storage.compute_returns(torch.randn(2 * B, 1, generator=torch.Generator().manual_seed(5)), 0.99, 0.95)
    idx = torch.randperm(T * 2 * B, generator=torch.Generator().manual_seed(4))[: T * B]
    st, ac = alg.storage, alg.actor_critic
    Bf = T * 2 * B
    ac.act(st.observations.view(Bf, -1)[idx])
    logp = ac.get_actions_log_prob(st.actions.view(Bf, -1)[idx])
    value = ac.evaluate(st.observations.view(Bf, -1)[idx])
    ratio = torch.exp(logp - st.actions_log_prob.view(Bf)[idx])
    adv = st.advantages.view(Bf)[idx]
    s_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.2)).mean()
    tv, ret = st.values.view(Bf, 1)[idx], st.returns.view(Bf, 1)[idx]
    vc = tv + (value - tv).clamp(-0.2, 0.2)
    v_loss = torch.max((value - ret).pow(2), (vc - ret).pow(2)).mean()
    (s_loss + v_loss - 0.01 * ac.entropy.mean()).backward()
    want = oracle_minibatch_grads(alg, idx)
    assert float(v_loss) == pytest.approx(want[0], rel=1e-5) and float(s_loss) == pytest.approx(want[1], rel=1e-5)
    worst, name = grad_deviation(ac, want[3], rtol=1e-4)
    assert worst <= 1.0, (worst, name)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, out_q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    alg = make_alg(B)
    fill(alg.storage, None, B, offset=rank * B)
    last = torch.randn(2 * B, 1, generator=torch.Generator().manual_seed(9))[rank * B:(rank + 1) * B]
    alg.storage.compute_returns(last, 0.99, 0.95, reduce_stats=alg._gather_moments)
    alg.update()
    if rank == 0:
        out_q.put([p.detach().numpy().copy() for p in alg.actor_critic.parameters()] + [alg.learning_rate])
    dist.barrier()
    dist.destroy_process_group()


def test_dp_advantage_statistics_are_chan_moments():
    """The data-parallel advantage statistics: per-rank float64 (count, mean, M2)
    summaries combined in rank order == the float64 mean / unbiased std of all samples, also when
    |mean| >> std (where sum / sum-of-squares in f32 collapses the variance)."""
    from legged_gym_amd.rl.storage import combined_mean_std, local_moments
    g = torch.Generator().manual_seed(5)
    for offset, scale in ((0.0, 1.0), (1.0e4, 1.0e-3), (-3.0e3, 0.5)):
        x = (offset + scale * torch.randn(4, 3000, 1, generator=g)).float()
        ranks = [x[:, :1000], x[:, 1000:1700], x[:, 1700:]]          # ragged shards
        mean, std = combined_mean_std(torch.cat([local_moments(r) for r in ranks]))
        xd = x.double().numpy().reshape(-1)
        assert mean == pytest.approx(xd.mean(), rel=1e-12, abs=1e-12)
        assert std == pytest.approx(xd.std(ddof=1), rel=1e-9)
    # the f32 sum / sum-of-squares form it replaces loses the large-mean case entirely
    xf = (1.0e4 + 1.0e-3 * torch.randn(12000, generator=g)).float()
    n = xf.numel()
    var_naive = float(((xf * xf).sum() - n * xf.mean() ** 2) / (n - 1))
    std_true = float(xf.double().std())
    assert abs(max(var_naive, 0.0) ** 0.5 - std_true) > 0.5 * std_true
    _, std = combined_mean_std(local_moments(xf))
    assert std == pytest.approx(std_true, rel=1e-9)


def test_data_parallel_equals_single_process_gloo():
    """2 ranks x B envs (gloo all-reduce of grads, global advantage stats, global KL) ==
    1 process x 2B envs, full-batch updates."""
    ref = make_alg(2 * B)
    fill(ref.storage, None, 2 * B)
    last = torch.randn(2 * B, 1, generator=torch.Generator().manual_seed(9))
    ref.storage.compute_returns(last, 0.99, 0.95)
    ref.update()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[-1] == pytest.approx(ref.learning_rate)
    for a, b in zip(got[:-1], ref.actor_critic.parameters()):
        np.testing.assert_allclose(a, b.detach().numpy(), rtol=1e-4, atol=2e-6)


def test_runner_learns_on_oracle_env_and_checkpoints(tmp_path):
    """End-to-end rsl_rl-style loop on the CPU oracle env: act -> step -> GAE -> update -> save/load."""
    from oracle_backend import make_env
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfgPPO
    env = make_env("go1_flat_bench", num_envs=8, device="cpu", backend="oracle")
    cfg = class_to_dict(Go1RoughCfgPPO())
    cfg["runner"]["num_steps_per_env"] = 4
    cfg["runner"]["save_interval"] = 1
    runner = OnPolicyRunner(env, cfg, str(tmp_path), device="cpu")
    runner.learn(2, init_at_random_ep_len=True)
    files = sorted(os.listdir(tmp_path))
    assert "model_0.pt" in files and "model_2.pt" in files
    runner.load(os.path.join(tmp_path, "model_2.pt"))
    assert runner.current_learning_iteration == 2
    pol = runner.get_inference_policy()
    with torch.inference_mode():
        a = pol(env.get_observations())
    assert a.shape == (8, 12) and torch.isfinite(a).all()


def test_runner_reports_the_original_error(tmp_path):
    """when learn() unwinds from an error, a failing cleanup (flush of the deferred
    storage row) must not replace the original exception, and no deferred row survives."""
    from oracle_backend import make_env
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfgPPO
    env = make_env("go1_flat_bench", num_envs=4, device="cpu", backend="oracle")
    cfg = class_to_dict(Go1RoughCfgPPO())
    cfg["runner"]["num_steps_per_env"] = 2
    runner = OnPolicyRunner(env, cfg, None, device="cpu")
    calls = {"n": 0}
    orig = env.step

    def failing_step(actions):
        calls["n"] += 1
        if calls["n"] == 2:
            runner.alg._pending_store = ("stale",)        # a deferred row whose flush will fail
            raise ValueError("env step failed")
        return orig(actions)

    def bad_flush():
        if runner.alg._pending_store is not None:
            raise RuntimeError("cleanup failed")
    env.step = failing_step
    runner.alg.flush_store = bad_flush
    with pytest.raises(ValueError, match="env step failed"):
        runner.learn(1)
    assert runner.alg._pending_store is None and runner.alg.defer_store is False


def test_policy_export_is_plain_torchscript(tmp_path):
    """helpers.py:180-190: the exported actor is a TorchScript module of plain layers."""
    from legged_gym_amd.utils import export_policy_as_jit
    torch.manual_seed(0)
    ac = ActorCritic(OBS, OBS, ACT, [16, 8], [16, 8])
    export_policy_as_jit(ac, str(tmp_path))
    pol = torch.jit.load(str(tmp_path / "policy_1.pt"))
    x = torch.randn(5, OBS)
    assert torch.allclose(pol(x), ac.actor(x), atol=1e-6)


@pytest.mark.parametrize("schedule", ["adaptive", "fixed"])
def test_resume_learning_rate_follows_upstream(tmp_path, schedule):
    """rsl_rl v1.0.x OnPolicyRunner.load restores the optimizer state only; alg.learning_rate keeps
    the config value.  Adaptive schedule: the first update after a resume adapts from the config
    value and writes it into the optimizer (the restored lr is overwritten); fixed schedule: the
    update steps with the restored optimizer lr."""
    from oracle_backend import make_env
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfgPPO
    env = make_env("go1_flat_bench", num_envs=8, device="cpu", backend="oracle")
    cfg = class_to_dict(Go1RoughCfgPPO())
    cfg["runner"]["num_steps_per_env"] = 4
    cfg["algorithm"]["schedule"] = schedule
    runner = OnPolicyRunner(env, cfg, None, device="cpu")
    for g in runner.alg.optimizer.param_groups:
        g["lr"] = 3.3e-4                           # a trained-run lr that differs from the config's
    path = str(tmp_path / "model_7.pt")
    runner.save(path)
    resumed = OnPolicyRunner(env, cfg, None, device="cpu")
    resumed.load(path)
    lr_cfg = cfg["algorithm"]["learning_rate"]
    assert resumed.alg.learning_rate == lr_cfg
    assert resumed.alg.optimizer.param_groups[0]["lr"] == 3.3e-4
    seen = []
    step = resumed.alg.optimizer.step

    def spy(*a, **k):
        seen.append(resumed.alg.optimizer.param_groups[0]["lr"])
        return step(*a, **k)
    resumed.alg.optimizer.step = spy
    resumed.learn(1)
    if schedule == "fixed":
        assert seen and all(lr == 3.3e-4 for lr in seen)
    else:   # adapted from the config value by factors of 1.5 (or kept), never the restored 3.3e-4
        # (clamped to [1e-5, 1e-2])
        ratios = [np.log(lr / lr_cfg) / np.log(1.5) for lr in seen if 1e-5 < lr < 1e-2]
        assert seen and ratios and all(abs(r - round(r)) < 1e-6 for r in ratios), seen
        assert 3.3e-4 not in seen


def test_play_logger(tmp_path):
    """utils/logger.py (legged_gym/utils/logger.py:36-136): reward bookkeeping weighted by episode
    counts, and the 3 x 3 state figure rendered headless."""
    from legged_gym_amd.utils.logger import Logger
    lg = Logger(0.02)
    for t in range(50):
        lg.log_states({"dof_pos": np.sin(t * 0.1), "dof_pos_target": 0.0, "dof_vel": 0.1 * t, "dof_torque": 1.0 - t,
                       "base_vel_x": 0.5, "command_x": 0.5, "contact_forces_z": np.array([1.0, 2.0, 3.0, 4.0])})
    lg.log_rewards({"rew_tracking": torch.tensor(2.0), "terrain_level": torch.tensor(3.0)}, 3)
    lg.log_rewards({"rew_tracking": torch.tensor(1.0)}, 1)
    assert lg.num_episodes == 4 and lg.average_rewards() == {"rew_tracking": (2.0 * 3 + 1.0) / 4}
    path = lg.plot_states(str(tmp_path / "s.png"))
    assert os.path.getsize(path) > 10000
