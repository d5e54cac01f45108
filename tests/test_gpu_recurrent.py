"""GPU: ActorCriticRecurrent's rollout - the LSTM on torch, its MLP heads on the fused rollout
kernel (lgx_mlp_x3_forward) - against the same policy evaluated on the CPU; one recurrent PPO update
on the autograd path (LGX_PPO_FUSED_RECURRENT=0); and the fused recurrent update (FusedPPOUpdate:
the memories on torch autograd, the heads on the fused kernels, dX = dZ_1 W_1 between them) checked
at every optimizer step against autograd (rl/ppo.py's recurrent update, legged_robot_config.py:221-224
names the rnn options)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_recurrent_rollout_heads_on_fused_kernel_match_cpu(gpu):
    from legged_gym_amd.rl.actor_critic import ActorCriticRecurrent
    from legged_gym_amd.rl.ppo import PPO
    torch.manual_seed(0)
    T, N, OBS, ACT = 4, 512, 48, 12
    ac_cpu = ActorCriticRecurrent(OBS, OBS, ACT, [512, 256, 128], [512, 256, 128], rnn_hidden_size=256)
    ac_gpu = copy.deepcopy(ac_cpu).to(gpu)
    gen = torch.Generator().manual_seed(1)
    obs = torch.randn(T, N, OBS, generator=gen)
    dones = torch.rand(T, N, generator=gen) < 0.2
    with torch.inference_mode():
        for t in range(T):
            _, v_c = ac_cpu.act_and_evaluate(obs[t], obs[t])
            mu_c = ac_cpu.action_mean
            _, v_g = ac_gpu.act_and_evaluate(obs[t].to(gpu), obs[t].to(gpu))
            mu_g = ac_gpu.action_mean
            assert ac_gpu._fused_actor.last_x3 is not None      # the heads ran on the fused kernel
            torch.testing.assert_close(mu_g.cpu(), mu_c, atol=2e-4, rtol=2e-4)
            torch.testing.assert_close(v_g.cpu(), v_c, atol=2e-4, rtol=2e-4)
            ac_cpu.reset(dones[t])
            ac_gpu.reset(dones[t].to(gpu))
    import os
    os.environ["LGX_PPO_FUSED_RECURRENT"] = "0"
    try:
        ppo = PPO(ac_gpu, num_learning_epochs=1, num_mini_batches=2, device=str(gpu))
    finally:
        del os.environ["LGX_PPO_FUSED_RECURRENT"]
    assert ppo._fused is None
    ppo.init_storage(N, T, [OBS], [None], [ACT])
    with torch.inference_mode():
        for t in range(T):
            ppo.act(obs[t].to(gpu), obs[t].to(gpu))
            ppo.process_env_step(torch.randn(N, device=gpu), dones[t].to(gpu), {})
        ppo.compute_returns(obs[-1].to(gpu))
    vl, sl = ppo.update()
    assert torch.isfinite(torch.tensor([vl, sl])).all()
    assert all(torch.isfinite(p).all() for p in ac_gpu.parameters())


def _recurrent_pair(gpu, T=8, N=512, OBS=48, ACT=12, hidden=(512, 256, 128), rnn=256, cobs=None, epochs=2):
    """Autograd and fused PPO on one ActorCriticRecurrent (deep copies), with identical storage
    filled by a rollout (saved LSTM states, dones mid-rollout) on the autograd one."""
    from legged_gym_amd.rl.actor_critic import ActorCriticRecurrent
    from legged_gym_amd.rl.ppo import PPO
    torch.manual_seed(0)
    ac = ActorCriticRecurrent(OBS, cobs or OBS, ACT, list(hidden), list(hidden), rnn_hidden_size=rnn).to(gpu)
    ac2 = copy.deepcopy(ac)
    kw = dict(num_learning_epochs=epochs, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95, value_loss_coef=1.0,
              entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0, schedule="adaptive", desired_kl=0.01,
              device=str(gpu))
    ref = PPO(ac, use_fused_update=False, **kw)
    fus = PPO(ac2, use_fused_update=True, **kw)
    assert ref._fused is None and fus._fused is not None and fus._fused.recurrent
    for p in (ref, fus):
        p.init_storage(N, T, [OBS], [cobs], [ACT])
    g = torch.Generator(device=gpu).manual_seed(4)
    with torch.inference_mode():
        for t in range(T):
            obs = torch.randn(N, OBS, device=gpu, generator=g)
            cob = torch.randn(N, cobs, device=gpu, generator=g) if cobs else obs
            ref.act(obs, cob)
            dones = torch.rand(N, device=gpu, generator=g) < 0.15
            ref.process_env_step(torch.randn(N, device=gpu, generator=g), dones, {})
        ref.compute_returns(torch.randn(N, cobs or OBS, device=gpu, generator=g))
    a, b = ref.storage, fus.storage
    for name in ("observations", "privileged_observations", "actions", "rewards", "dones", "values", "returns",
                 "advantages", "actions_log_prob", "mu", "sigma"):
        if getattr(a, name) is not None:
            getattr(b, name).copy_(getattr(a, name))
    b.saved_hidden_states_a = [h.clone() for h in a.saved_hidden_states_a]
    b.saved_hidden_states_c = [h.clone() for h in a.saved_hidden_states_c]
    b.step = a.step
    return ref, fus


def _autograd_minibatch_grads(ref, batch):
    """rl/ppo.py's recurrent loss of one minibatch (the generator's tuple) at ref's current
    parameters: {name: grad}."""
    obs_b, cobs_b, act_b, target_v_b, adv_b, ret_b, old_logp_b, old_mu_b, old_sigma_b, hid_b, masks_b = batch
    ac = ref.actor_critic
    ac.act(obs_b, masks=masks_b, hidden_states=hid_b[0])
    logp_b = ac.get_actions_log_prob(act_b)
    value_b = ac.evaluate(cobs_b, masks=masks_b, hidden_states=hid_b[1])
    ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
    adv = torch.squeeze(adv_b)
    s = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.2)).mean()
    vc = target_v_b + (value_b - target_v_b).clamp(-0.2, 0.2)
    vl = torch.max((value_b - ret_b).pow(2), (vc - ret_b).pow(2)).mean()
    loss = s + vl - 0.01 * ac.entropy.mean()
    for p in ac.parameters():
        p.grad = None
    loss.backward()
    return {n: p.grad.detach().clone() for n, p in ac.named_parameters()}


@pytest.mark.parametrize("cobs,rnn", [(None, 256), (60, 72)])
def test_fused_recurrent_update_every_step_matches_autograd(gpu, cobs, rnn):
    """Every optimizer step of the fused recurrent update (2 epochs x 4 minibatches of whole-env
    trajectories): the flat gradient it consumed (heads from the fused kernels, memories from
    autograd fed with dX = dZ_1 W_1) == autograd's at the recorded parameters and minibatch,
    |d| <= 1e-5 + 2e-3 |g|; the step == float64 clip + Adam of that gradient; the learning-rate
    sequence identical.  rnn = 72: the heads' input is copied into rows padded to the GEMM's K step
    (96) and dW1 leaves lgx_gemm_tn (library bmm); cobs: a critic memory over privileged observations."""
    from ppo_trace import StepTrace, adam64, flat_view
    ref, fus = _recurrent_pair(gpu, cobs=cobs, rnn=rnn)
    f = fus._fused
    batches = list(ref.storage.reccurent_mini_batch_generator(4, 2))
    tr = StepTrace(f)
    vl_f, sl_f = fus.update()
    tr.close()
    vl_r, sl_r = ref.update()
    assert fus.learning_rate == ref.learning_rate
    assert abs(vl_f - vl_r) <= 1e-4 * abs(vl_r) + 1e-6 and abs(sl_f - sl_r) <= 1e-4 * abs(sl_r) + 1e-6
    assert len(tr.steps) == len(batches) == 8
    params = list(ref.actor_critic.parameters())
    for t, rec in enumerate(tr.steps):
        with torch.no_grad():
            for p, q in zip(params, f.optimizer.params):
                off = f.off[id(q)]
                p.copy_(rec["p0"][off:off + q.numel()].view_as(p))
        g_ref = flat_view(f, list(_autograd_minibatch_grads(ref, batches[t]).values()))
        g = rec["g"].double()
        bad = ((g - g_ref).abs() > 1e-5 + 2e-3 * g_ref.abs()).sum().item()
        assert bad == 0, (t, bad, (g - g_ref).abs().max().item())
        mem = slice(f.off[id(f.mem_params[0])], f.n)        # the memories' block is not zero
        assert g_ref[mem].abs().max() > 0 and g[mem].abs().max() > 0
        p_want, _, _ = adam64(rec, fus.max_grad_norm)
        dp = (rec["p1"].double() - p_want).abs()
        assert (dp <= 1e-6 + 1e-3 * rec["lr"]).all(), (t, dp.max().item())
