"""PPO with the rsl_rl v1.0.x algorithm and hyper-parameter contract
(legged_robot_config.py:226-239; upstream rsl_rl `PPO`), data-parallel over ranks.

Data parallelism (new; the reference is single-GPU): every rank owns its envs and a full
ActorCritic replica.  Per minibatch the flat fp32 gradient is all-reduced (RCCL over xGMI when
the process group backend is "nccl") and averaged before clip_grad_norm, advantage
normalisation uses global statistics, and the KL used by the adaptive learning rate is the
global mean, so every rank applies the identical Adam step and N ranks x B envs reproduce
1 rank x N*B envs up to reduction order.
"""
import ctypes as C

import os

import torch
import torch.nn as nn
import torch.optim as optim

from legged_gym_amd.sim import abi

from .actor_critic import ActorCritic, launch_forward, make_descs
from .fused_ppo import FusedPPOUpdate
from .storage import RolloutStorage


def _dist():
    """torch.distributed when the job runs data-parallel (world > 1).  LGX_DIST_REHEARSAL=1 takes the
    data-parallel path at world 1 too (every collective over a one-rank RCCL communicator): the
    single-GPU rehearsal of the multi-GPU code path (bench.py, tests/test_gpu_ddp.py)."""
    import os
    import torch.distributed as dist
    least = 1 if os.environ.get("LGX_DIST_REHEARSAL") == "1" else 2
    return dist if dist.is_available() and dist.is_initialized() and dist.get_world_size() >= least else None


class PPO:
    actor_critic: ActorCritic

    def __init__(self, actor_critic, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998, lam=0.95,
                 value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu", use_fused_update=True):
        self.device = device
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.learning_rate = learning_rate
        self.actor_critic = actor_critic.to(self.device)
        self.storage = None
        fused = str(device).startswith("cuda")
        self.optimizer = optim.Adam(self.actor_critic.parameters(), lr=learning_rate, fused=fused or None)
        self.transition = RolloutStorage.Transition()
        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.dist = _dist()
        self._fused = None
        # process_env_step leaves its storage-row launch to the next act (one launch per step);
        # set by OnPolicyRunner, whose loop always calls act between env.step calls
        self.defer_store = False
        self._pending_store = None
        if fused and use_fused_update and FusedPPOUpdate.supported(self.actor_critic):
            self._fused = FusedPPOUpdate(self)       # parameters become views of its flat buffer
            self.optimizer = self._fused.optimizer
        if self.dist is not None:
            self._broadcast_params()

    # ---------------------------------------------------------------- setup / modes
    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                                      action_shape, self.device)

    def test_mode(self):
        self.actor_critic.test()

    def train_mode(self):
        self.actor_critic.train()

    def _broadcast_params(self):
        with torch.no_grad():
            for p in self.actor_critic.parameters():
                self.dist.broadcast(p.data, src=0)

    # ---------------------------------------------------------------- rollout
    def _rollout_kernels_ok(self, obs):
        ac = self.actor_critic
        return (self._fused is not None and obs.is_cuda and self.storage is not None
                and getattr(ac, "rollout_forward", None) is not None and not ac.is_recurrent
                and self.storage.step < self.storage.num_transitions_per_env)

    def _act_fused(self, obs, critic_obs):
        """act() + add_transitions' row writes (+ the deferred process_env_step store of the previous
        step) in ONE launch: lgx_mlp_x3_forward_act runs the actor and critic MLPs and lgx_ppo_act's
        arithmetic in the actor's last-layer epilogue (the critic writes its storage row directly).
        LGX_FUSED_ACT=0, or a network pair the fused launch does not take: the MLP launch, then
        lgx_ppo_act(_store) - bit-identical rows either way."""
        ac = self.actor_critic
        if not (ac._fused_ok(obs, ac._fused_actor) and ac._fused_critic.ok):
            return None
        st, s = self.storage, self.storage.step
        main = torch.cuda.current_stream(obs.device)
        obs = obs.contiguous()
        critic_obs = critic_obs.contiguous()
        A = ac._fused_actor.dims[-1]
        if getattr(self, "_mean_buf", None) is None or self._mean_buf.shape != (obs.shape[0], A):
            self._mean_buf = torch.empty(obs.shape[0], A, device=obs.device)
        mean = self._mean_buf
        descs = make_descs([(ac._fused_actor, obs, mean), (ac._fused_critic, critic_obs, st.values[s])])
        if getattr(self, "_act_out", None) is None or self._act_out.shape != mean.shape:
            self._act_out = torch.empty_like(mean)
        # Normal.sample's standard-normal draws from torch's generator.  Default: one [N, A] draw
        # per step, the RNG consumption of rsl_rl's Normal.sample (torch.normal(mu, std) =
        # normal_(0, 1) * std + mu), so seeded runs draw the same noise as upstream.
        # LGX_BATCHED_NOISE=1: one [T, N, A] draw per rollout (one launch instead of T; same
        # distribution, different RNG stream, T*N*A floats kept)
        T = st.num_transitions_per_env
        if os.environ.get("LGX_BATCHED_NOISE", "0") == "1":
            if s == 0 or getattr(self, "_noise", None) is None or self._noise.shape != (T,) + tuple(mean.shape):
                self._noise = torch.randn((T,) + tuple(mean.shape), device=mean.device)
            noise = self._noise[s]
        else:
            noise = torch.randn(mean.shape, device=mean.device)
            self._noise = noise   # keep it alive until the act kernel has read it
        a = abi.LgxPpoActArgs()
        a.num_envs, a.num_actions, a.num_obs = mean.shape[0], mean.shape[1], obs.shape[1]
        a.mu, a.value, a.std, a.noise = mean.data_ptr(), None, self.actor_critic.std.data_ptr(), noise.data_ptr()
        a.obs = obs.data_ptr()
        if st.privileged_observations is not None:
            a.num_cobs, a.cobs, a.st_cobs = critic_obs.shape[1], critic_obs.data_ptr(), \
                st.privileged_observations[s].data_ptr()
        a.actions_out = self._act_out.data_ptr()
        a.st_obs, a.st_actions, a.st_values = st.observations[s].data_ptr(), st.actions[s].data_ptr(), \
            st.values[s].data_ptr()
        a.st_logp, a.st_mu, a.st_sigma = st.actions_log_prob[s].data_ptr(), st.mu[s].data_ptr(), st.sigma[s].data_ptr()
        lib = self._fused.lib
        stream = C.c_void_p(main.cuda_stream)
        pend = getattr(self, "_pending_store", None)
        prev = pend[0] if pend is not None and pend[0].num_envs == a.num_envs else None
        if prev is None:
            self.flush_store()
        fused = (isinstance(descs[0], abi.LgxMlpX3Desc) and not getattr(self, "_fused_act_off", False)
                 and os.environ.get("LGX_FUSED_ACT", "1") != "0")
        if fused and lib.lgx_mlp_x3_forward_act(descs, 2, C.byref(a), C.byref(prev) if prev is not None else None,
                                                stream) != 0:
            # (validated before any launch) a pair the fused launch does not take, e.g. the act
            # rows past the LDS: the two-launch form from now on
            self._fused_act_off, fused = True, False
        if not fused:
            launch_forward(descs, 2, stream)   # actor and critic in one launch
            if prev is not None:   # the previous step's store rides along
                self._fused.check(lib.lgx_ppo_act_store(C.byref(a), C.byref(prev), stream), "lgx_ppo_act_store")
            else:
                self._fused.check(lib.lgx_ppo_act(C.byref(a), stream), "lgx_ppo_act")
        self.last_act_fused = fused
        if prev is not None:
            self._pending_store = None
        t = self.transition
        t.actions, t.values = self._act_out, st.values[s]
        t.actions_log_prob, t.action_mean, t.action_sigma = st.actions_log_prob[s], st.mu[s], st.sigma[s]
        t.observations, t.critic_observations = obs, critic_obs
        t.in_storage = True
        return self._act_out

    def act(self, obs, critic_obs):
        t = self.transition
        if self._rollout_kernels_ok(obs):
            actions = self._act_fused(obs, critic_obs)
            if actions is not None:
                return actions
        self.flush_store()   # (a deferred store reads the env's buffers before the next env.step)
        if self.actor_critic.is_recurrent:   # the memories' state before this step (rsl_rl PPO.act)
            t.hidden_states = self.actor_critic.get_hidden_states()
        if hasattr(self.actor_critic, "act_and_evaluate"):
            actions, values = self.actor_critic.act_and_evaluate(obs, critic_obs)
            t.actions, t.values = actions.detach(), values.detach()
        else:
            t.actions = self.actor_critic.act(obs).detach()
            t.values = self.actor_critic.evaluate(critic_obs).detach()
        t.actions_log_prob = self.actor_critic.get_actions_log_prob(t.actions).detach()
        t.action_mean = self.actor_critic.action_mean.detach()
        t.action_sigma = self.actor_critic.action_std.detach()
        t.observations = obs
        t.critic_observations = critic_obs
        return t.actions

    def process_env_step(self, rewards, dones, infos):
        t = self.transition
        if getattr(t, "in_storage", False):     # row already written by lgx_ppo_act
            st = self.storage
            a = abi.LgxPpoStoreArgs()
            a.num_envs, a.gamma = st.num_envs, self.gamma
            rewards = rewards.contiguous()
            dones = dones.contiguous()
            a.rew, a.reset = rewards.data_ptr(), dones.data_ptr()
            to = infos.get("time_outs") if isinstance(infos, dict) else None
            if to is not None:
                to = to.contiguous()
                a.time_outs = to.data_ptr()
            a.st_values, a.st_rew, a.st_dones = st.values[st.step].data_ptr(), st.rewards[st.step].data_ptr(), \
                st.dones[st.step].data_ptr()
            if self.defer_store:
                # launched with the next act (lgx_ppo_act_store) or by flush_store(): the env's
                # reward / reset / time-out buffers hold this step's values until the next env.step,
                # which the runner issues only after that act
                self.flush_store()
                self._pending_store = (a, rewards, dones, to)
            else:
                self._fused.check(self._fused.lib.lgx_ppo_store(C.byref(a), C.c_void_p(
                    torch.cuda.current_stream(rewards.device).cuda_stream)), "lgx_ppo_store")
            st.step += 1
            t.clear()
            self.actor_critic.reset(dones)
            return
        t.rewards = rewards.clone()
        t.dones = dones
        if "time_outs" in infos:  # bootstrap on time-outs
            t.rewards += self.gamma * torch.squeeze(t.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(t)
        t.clear()
        self.actor_critic.reset(dones)

    def flush_store(self):
        """Launch a deferred lgx_ppo_store (defer_store) on its own."""
        pend = getattr(self, "_pending_store", None)
        if pend is None:
            return
        self._pending_store = None
        self._fused.check(self._fused.lib.lgx_ppo_store(C.byref(pend[0]), C.c_void_p(
            torch.cuda.current_stream(pend[1].device).cuda_stream)), "lgx_ppo_store")

    def _gather_moments(self, parts):
        """Every rank's flat float64 (count, mean, M2) advantage summaries, concatenated in rank order
        (all_gather: identical on every rank, so every rank normalises with the same statistics)."""
        parts = parts.contiguous()
        if self.dist is None:
            return parts
        out = [torch.empty_like(parts) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(out, parts)
        return torch.cat(out)

    def compute_returns(self, last_critic_obs):
        self.flush_store()
        last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam,
                                     reduce_stats=self._gather_moments if self.dist is not None else None)

    # ---------------------------------------------------------------- update
    def _allreduce_grads(self):
        params = [p for p in self.actor_critic.parameters() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        self.dist.all_reduce(flat)
        flat /= self.dist.get_world_size()
        off = 0
        for p in params:
            n = p.grad.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n

    def update(self, defer=False):
        """rsl_rl PPO.update -> (mean value loss, mean surrogate loss).  defer=True (fused path only)
        issues the update and returns None; resolve() returns the losses later (FusedPPOUpdate)."""
        self.flush_store()
        if self._fused is not None:
            out = self._fused.update(defer=defer)
            self.storage.clear()
            if hasattr(self.actor_critic, "invalidate_fused"):
                self.actor_critic.invalidate_fused()
            return out
        mean_value_loss = 0.0
        mean_surrogate_loss = 0.0
        if self.actor_critic.is_recurrent:
            gen = self.storage.reccurent_mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        else:
            gen = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        for (obs_b, cobs_b, act_b, target_v_b, adv_b, ret_b, old_logp_b, old_mu_b, old_sigma_b, hid_b, masks_b) in gen:
            self.actor_critic.act(obs_b, masks=masks_b, hidden_states=hid_b[0])
            logp_b = self.actor_critic.get_actions_log_prob(act_b)
            value_b = self.actor_critic.evaluate(cobs_b, masks=masks_b, hidden_states=hid_b[1])
            mu_b = self.actor_critic.action_mean
            sigma_b = self.actor_critic.action_std
            entropy_b = self.actor_critic.entropy
            if self.desired_kl is not None and self.schedule == "adaptive":
                with torch.inference_mode():
                    kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1.e-5) +
                                   (torch.square(old_sigma_b) + torch.square(old_mu_b - mu_b)) /
                                   (2.0 * torch.square(sigma_b)) - 0.5, axis=-1)
                    kl_mean = torch.mean(kl)
                    if self.dist is not None:
                        self.dist.all_reduce(kl_mean)
                        kl_mean /= self.dist.get_world_size()
                    kl_mean = kl_mean.item()
                    if kl_mean > self.desired_kl * 2.0:
                        self.learning_rate = max(1e-5, self.learning_rate / 1.5)
                    elif self.desired_kl / 2.0 > kl_mean > 0.0:
                        self.learning_rate = min(1e-2, self.learning_rate * 1.5)
                    for g in self.optimizer.param_groups:
                        g["lr"] = self.learning_rate
            ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
            adv = torch.squeeze(adv_b)
            surrogate = -adv * ratio
            surrogate_clipped = -adv * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
            surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
            if self.use_clipped_value_loss:
                value_clipped = target_v_b + (value_b - target_v_b).clamp(-self.clip_param, self.clip_param)
                value_loss = torch.max((value_b - ret_b).pow(2), (value_clipped - ret_b).pow(2)).mean()
            else:
                value_loss = (ret_b - value_b).pow(2).mean()
            loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_b.mean()
            self.optimizer.zero_grad()
            loss.backward()
            if self.dist is not None:
                self._allreduce_grads()
            nn.utils.clip_grad_norm_(self.actor_critic.parameters(), self.max_grad_norm)
            self.optimizer.step()
            mean_value_loss += value_loss.detach()
            mean_surrogate_loss += surrogate_loss.detach()
        if hasattr(self.actor_critic, "invalidate_fused"):
            self.actor_critic.invalidate_fused()
        n = self.num_learning_epochs * self.num_mini_batches
        mean_value_loss = (mean_value_loss / n).item()
        mean_surrogate_loss = (mean_surrogate_loss / n).item()
        self.storage.clear()
        if defer:
            self._deferred = (mean_value_loss, mean_surrogate_loss)
            return None
        return mean_value_loss, mean_surrogate_loss

    def resolve(self):
        """The losses of an update(defer=True) (applying the fused path's learning-rate readback),
        or None when none is pending."""
        if self._fused is not None:
            return self._fused.resolve()
        out, self._deferred = getattr(self, "_deferred", None), None
        return out
