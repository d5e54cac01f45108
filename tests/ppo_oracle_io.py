"""Test helper: run oracle/ppo_oracle.py (numpy float64 restatement of rsl_rl's PPO.update) on a
PPO instance's storage / parameters, and compare an updated ActorCritic against its result."""
import importlib.util
import os

import numpy as np
import torch
import torch.nn as nn

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("ppo_oracle", os.path.join(_ROOT, "oracle", "ppo_oracle.py"))
ppo_oracle = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(ppo_oracle)


def _lin(seq):
    return [(m.weight.detach().double().cpu().numpy(), m.bias.detach().double().cpu().numpy())
            for m in seq if isinstance(m, nn.Linear)]


def _batch(alg):
    st = alg.storage
    f = lambda t: t.detach().double().flatten(0, 1).cpu().numpy()   # time-major rows, as the generator
    obs = f(st.observations)
    return dict(obs=obs, cobs=f(st.privileged_observations) if st.privileged_observations is not None else obs,
                actions=f(st.actions), values=f(st.values), advantages=f(st.advantages), returns=f(st.returns),
                logp=f(st.actions_log_prob), mu=f(st.mu), sigma=f(st.sigma))


def oracle_minibatch_grads(alg, idx):
    """(value_loss, surrogate_loss, kl_mean, grads) of the minibatch rows idx (flattened
    time-major storage rows) at alg's current parameters; grads in _ordered() order."""
    ac = alg.actor_critic
    return ppo_oracle.minibatch_grads(_lin(ac.actor), _lin(ac.critic), ac.std.detach().double().cpu().numpy(),
                                      _batch(alg), np.asarray(idx.cpu().numpy()), alg.clip_param, alg.value_loss_coef,
                                      alg.entropy_coef, alg.use_clipped_value_loss)


def grad_deviation(ac, want_grads, rtol):
    """Largest |grad - oracle| / (1e-5 + rtol |oracle|) over the parameters (<= 1 passes), with
    the parameter's name."""
    worst, name = 0.0, None
    for (n, p), w in zip(_ordered(ac), want_grads):
        r = float(np.max(np.abs(p.grad.detach().double().cpu().numpy() - w) / (1e-5 + rtol * np.abs(w))))
        if r > worst:
            worst, name = r, n
    return worst, name


def _ordered(ac):
    """(name, parameter) in the oracle's order: actor (W, b) per layer, critic (W, b), std."""
    out = []
    for tag, seq in (("actor", ac.actor), ("critic", ac.critic)):
        for i, m in enumerate(seq):
            if isinstance(m, nn.Linear):
                out += [(f"{tag}.{i}.weight", m.weight), (f"{tag}.{i}.bias", m.bias)]
    return out + [("std", ac.std)]


def oracle_update(alg, seed):
    """The oracle's update of `alg` (same storage, same parameters, the permutation that
    torch.randperm draws after torch.manual_seed(seed) on the storage's device).  Call before
    alg.update(), which must then be preceded by torch.manual_seed(seed) too."""
    st = alg.storage
    batch = _batch(alg)
    B = st.num_envs * st.num_transitions_per_env
    nmb = alg.num_mini_batches
    torch.manual_seed(seed)
    perm = torch.randperm(nmb * (B // nmb), device=st.observations.device).cpu().numpy()
    ac = alg.actor_critic
    return ppo_oracle.ppo_update(_lin(ac.actor), _lin(ac.critic), ac.std.detach().double().cpu().numpy(), batch, perm,
                                 alg.num_learning_epochs, nmb, alg.learning_rate, clip_param=alg.clip_param,
                                 value_loss_coef=alg.value_loss_coef, entropy_coef=alg.entropy_coef,
                                 max_grad_norm=alg.max_grad_norm, desired_kl=alg.desired_kl, schedule=alg.schedule,
                                 use_clipped_value_loss=alg.use_clipped_value_loss)


def param_deviation(ac, oracle_out):
    """(max |d|, number of coordinates with |d| > 1e-5, total coordinates) of the updated
    ActorCritic against the oracle's parameters."""
    actor, critic, std = oracle_out[:3]
    want = [a for wb in actor for a in wb] + [a for wb in critic for a in wb] + [std]
    got = [p for _, p in _ordered(ac)]
    dmax, big, total = 0.0, 0, 0
    for g, w in zip(got, want):
        d = np.abs(g.detach().double().cpu().numpy() - w)
        dmax = max(dmax, float(d.max()))
        big += int((d > 1e-5).sum())
        total += d.size
    return dmax, big, total
