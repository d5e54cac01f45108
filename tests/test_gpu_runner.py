"""GPU: one OnPolicyRunner.learn iteration (rsl_rl v1.0.x semantics, the loop scripts/train.py:43
runs: task_registry.py:159-167) on the HIP path - fused rollout kernels, lgx_step, lgx_gae, the
fused PPO update - recorded as it runs and checked step by step against the reference semantics
evaluated independently in torch:
  * init_at_random_ep_len: episode_length_buf = randint_like(high=max_episode_length) with the
    caller's RNG state;
  * collection order act -> env.step -> process_env_step: storage row t holds the observation
    the policy acted on (bitwise), its actions (bitwise), value / mean / sigma / log-prob of the
    pre-update policy (torch fp32 modules), reward + gamma V time_outs (time-out bootstrap) and
    the done flags; the next act sees the observation env.step returned (bitwise);
  * GAE + advantage normalisation from the stored rows and the last critic value (torch loop);
  * the update == the autograd PPO.update (rl/ppo.py, pinned on CPU against the numpy oracle) on
    the same storage, parameters and RNG state: losses, learning-rate sequence, parameters
    (all but <= 0.1 % of the coordinates within 1e-5; every coordinate of every step is checked
    in test_gpu_ppo.py::test_fused_update_every_step_is_exact);
  * checkpoint cadence: model_<it>.pt every save_interval iterations plus the final one, in the
    rsl_rl dict format.
Tolerances: split-bf16 / f32 MFMA vs torch f32: values / means 2e-4; log-prob 1e-3 abs.
"""
import copy
import os

import pytest
import torch
from torch.distributions import Normal

from oracle_backend import make_env

pytestmark = pytest.mark.gpu


def test_runner_iteration_matches_reference_semantics(gpu, tmp_path):
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfgPPO
    from legged_gym_amd.rl.ppo import PPO
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    N = 512
    env = make_env("go1_rough", num_envs=N, device="cuda:0", backend="lgx")
    cfg = class_to_dict(Go1RoughCfgPPO())
    cfg["runner"]["save_interval"] = 1
    T = cfg["runner"]["num_steps_per_env"]
    torch.manual_seed(0)
    runner = OnPolicyRunner(env, cfg, str(tmp_path), device="cuda:0")
    alg = runner.alg
    assert alg._fused is not None
    ac0 = copy.deepcopy(alg.actor_critic)           # the pre-update policy (torch modules)
    rec = {"steps": []}
    orig_act, orig_step, orig_update, orig_gae = alg.act, env.step, alg.update, alg.compute_returns

    def act(obs, cobs):
        a = orig_act(obs, cobs)
        rec["steps"].append({"obs": obs.clone(), "actions": a.clone()})
        return a

    def env_step(actions):
        if len(rec["steps"]) == 1:
            rec["ep_len0"] = env._episode_length_buf.clone()
        out = orig_step(actions)
        rec["steps"][-1].update(next_obs=out[0].clone(), rew=out[2].clone(), done=out[3].clone(),
                                time_outs=out[4]["time_outs"].clone())
        return out

    def gae(last_critic_obs):
        rec["last_obs"] = last_critic_obs.clone()
        st = alg.storage
        rec["pre_gae"] = {k: getattr(st, k).clone() for k in ("rewards", "values", "dones")}
        return orig_gae(last_critic_obs)

    def update():
        st = alg.storage
        rec["storage"] = {k: getattr(st, k).clone() for k in ("observations", "actions", "rewards", "dones", "values",
                                                            "actions_log_prob", "mu", "sigma", "returns", "advantages")}
        rec["rng"] = (torch.get_rng_state(), torch.cuda.get_rng_state())
        rec["lr0"] = alg.learning_rate
        rec["params0"] = [p.detach().clone() for p in alg.actor_critic.parameters()]
        rec["losses"] = orig_update()
        return rec["losses"]

    alg.act, env.step, alg.update, alg.compute_returns = act, env_step, update, gae
    torch.manual_seed(123)
    runner.learn(1, init_at_random_ep_len=True)

    # init_at_random_ep_len
    torch.manual_seed(123)
    want = torch.randint_like(env._episode_length_buf, high=int(env.max_episode_length))
    assert torch.equal(rec["ep_len0"], want)
    # collection
    steps, st = rec["steps"], rec["storage"]
    assert len(steps) == T
    for t, s in enumerate(steps):
        assert torch.equal(st["observations"][t], s["obs"]), t
        assert torch.equal(st["actions"][t], s["actions"]), t
        if t + 1 < T:
            assert torch.equal(steps[t + 1]["obs"], s["next_obs"]), t
        with torch.no_grad():
            mu, v = ac0.actor(s["obs"]), ac0.critic(s["obs"])
        assert torch.allclose(st["mu"][t], mu, atol=2e-4, rtol=2e-4), t
        assert torch.allclose(rec["pre_gae"]["values"][t], v, atol=2e-4, rtol=2e-4), t
        assert torch.equal(st["sigma"][t], ac0.std.detach().expand_as(mu)), t
        logp = Normal(st["mu"][t], st["sigma"][t]).log_prob(s["actions"]).sum(-1)
        assert torch.allclose(st["actions_log_prob"][t, :, 0], logp, atol=1e-3, rtol=1e-5), t
        boot = s["rew"] + alg.gamma * rec["pre_gae"]["values"][t, :, 0] * s["time_outs"].float()
        assert torch.allclose(rec["pre_gae"]["rewards"][t, :, 0], boot, atol=1e-6, rtol=1e-6), t
        assert torch.equal(rec["pre_gae"]["dones"][t, :, 0], s["done"].to(torch.uint8)), t
    # GAE + normalisation (torch loop over the stored rows)
    with torch.no_grad():
        last = ac0.critic(rec["last_obs"])
    r, v, d = (rec["pre_gae"][k].double() for k in ("rewards", "values", "dones"))
    ret = torch.zeros_like(r)
    adv = torch.zeros_like(r[0])
    for t in reversed(range(T)):
        nv = last.double() if t == T - 1 else v[t + 1]
        nt = 1.0 - d[t]
        delta = r[t] + nt * alg.gamma * nv - v[t]
        adv = delta + nt * alg.gamma * alg.lam * adv
        ret[t] = adv + v[t]
    a = ret - v
    a = (a - a.mean()) / (a.std() + 1e-8)
    assert torch.allclose(st["returns"].double(), ret, atol=1e-4, rtol=1e-5)
    assert torch.allclose(st["advantages"].double(), a, atol=1e-4, rtol=1e-4)
    # the update against the autograd PPO on the same storage / parameters / RNG state
    ac_ref = copy.deepcopy(ac0)
    with torch.no_grad():
        for p, q in zip(ac_ref.parameters(), rec["params0"]):
            p.copy_(q)
    alg_cfg = dict(cfg["algorithm"])
    ref = PPO(ac_ref, device="cuda:0", use_fused_update=False, **alg_cfg)
    ref.learning_rate = rec["lr0"]
    ref.init_storage(N, T, [env.num_obs], [None], [env.num_actions])
    for k, val in st.items():
        getattr(ref.storage, k).copy_(val)
    ref.storage.step = T
    torch.set_rng_state(rec["rng"][0])
    torch.cuda.set_rng_state(rec["rng"][1])
    vl, sl = ref.update()
    assert alg.learning_rate == ref.learning_rate
    assert abs(rec["losses"][0] - vl) <= 1e-4 * abs(vl) + 1e-6 and abs(rec["losses"][1] - sl) <= 1e-4 * abs(sl) + 1e-6
    big = total = 0
    for p, q in zip(alg.actor_critic.parameters(), ac_ref.parameters()):
        dd = (p - q).abs()
        big += int((dd > 1e-5).sum())
        total += dd.numel()
    assert big <= 1e-3 * total, (big, total)
    # checkpoint cadence (save_interval 1: iteration 0, then the final model_1.pt)
    files = sorted(f for f in os.listdir(tmp_path) if f.endswith(".pt"))
    assert files == ["model_0.pt", "model_1.pt"], files
    ck = torch.load(tmp_path / "model_1.pt", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "iter", "infos"} and ck["iter"] == 1
    for k, p in alg.actor_critic.state_dict().items():
        assert torch.equal(ck["model_state_dict"][k], p), k


@pytest.mark.parametrize("defer_store", ["1", "0"])
def test_deferred_readback_matches_synchronous_runner(gpu, tmp_path, monkeypatch, defer_store):
    """learn() without a log directory issues each update with a deferred readback (the
    statistics are taken after the next rollout is issued); with one it reads them back at once.
    Same seeds, 3 iterations each: identical parameters, Adam moments, learning rate and final
    iteration statistics (bitwise: the same kernels in the same order).  The synchronous run keeps
    every step's storage store in its own launch (LGX_DEFER_STORE=0); the deferred run rides it on
    the next act's launch (lgx_ppo_act_store) or not (parametrized)."""
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfgPPO
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    out = []
    for log_dir in (None, str(tmp_path)):
        monkeypatch.setenv("LGX_DEFER_STORE", defer_store if log_dir is None else "0")
        env = make_env("go1_rough", num_envs=256, device="cuda:0", backend="lgx")
        cfg = class_to_dict(Go1RoughCfgPPO())
        cfg["runner"]["save_interval"] = 100
        torch.manual_seed(0)
        runner = OnPolicyRunner(env, cfg, log_dir, device="cuda:0")
        deferred = []
        orig = runner.alg.update
        runner.alg.update = lambda defer=False: (deferred.append(defer), orig(defer=defer))[1]
        torch.manual_seed(7)
        runner.learn(3, init_at_random_ep_len=True)
        torch.cuda.synchronize()
        assert deferred == [log_dir is None] * 3
        assert runner.alg._fused._pending is None
        o = runner.alg.optimizer
        out.append(([p.detach().clone() for p in runner.alg.actor_critic.parameters()],
                    o.m.clone(), o.v.clone(), runner.alg.learning_rate, o.param_groups[0]["lr"],
                    {k: v for k, v in runner.last_iteration_stats.items() if k.endswith("loss") or k == "learning_rate"}))
    (pa, ma, va, lra, pga, sa), (pb, mb, vb, lrb, pgb, sb) = out
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    assert torch.equal(ma, mb) and torch.equal(va, vb)
    assert lra == lrb and pga == pgb and sa == sb, (lra, lrb, sa, sb)
