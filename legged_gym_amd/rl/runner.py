"""OnPolicyRunner with the rsl_rl v1.0.x contract consumed by the reference
(task_registry.py:159-167, train.py:43, play.py:65-71): `OnPolicyRunner(env, train_cfg_dict,
log_dir, device)`, `learn(num_learning_iterations, init_at_random_ep_len)`, `save`, `load`,
`get_inference_policy`, `alg.actor_critic`; checkpoint dict {model_state_dict,
optimizer_state_dict, iter, infos} saved every `save_interval` iterations as model_<it>.pt.

Timing: `collection_time` (act + env.step + storage) and `learn_time` (GAE + update) per
iteration, fps = num_steps_per_env * num_envs / (collection + learn), as rsl_rl logs it;
`last_iteration_stats` keeps them for bench.py.
"""
import os
import statistics
import time
from collections import deque

import torch

from .actor_critic import ActorCritic, ActorCriticRecurrent  # noqa: F401  (resolved by name from the cfg)
from .ppo import PPO  # noqa: F401


class OnPolicyRunner:
    def __init__(self, env, train_cfg, log_dir=None, device="cpu"):
        self.cfg = train_cfg["runner"]
        self.alg_cfg = train_cfg["algorithm"]
        self.policy_cfg = train_cfg["policy"]
        self.device = device
        self.env = env
        num_critic_obs = self.env.num_privileged_obs if self.env.num_privileged_obs is not None else self.env.num_obs
        ac_class = {"ActorCritic": ActorCritic,
                    "ActorCriticRecurrent": ActorCriticRecurrent}[self.cfg["policy_class_name"]]
        actor_critic = ac_class(self.env.num_obs, num_critic_obs, self.env.num_actions, **self.policy_cfg).to(self.device)
        alg_class = {"PPO": PPO}[self.cfg["algorithm_class_name"]]
        self.alg = alg_class(actor_critic, device=self.device, **self.alg_cfg)
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        self.alg.init_storage(self.env.num_envs, self.num_steps_per_env, [self.env.num_obs],
                              [self.env.num_privileged_obs], [self.env.num_actions])
        self.log_dir = log_dir
        self.writer = None
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.last_iteration_stats = {}
        _, _ = self.env.reset()

    def _writer(self):
        if self.writer is None and self.log_dir is not None:
            try:
                from torch.utils.tensorboard import SummaryWriter
                self.writer = SummaryWriter(log_dir=self.log_dir, flush_secs=10)
            except Exception:
                self.writer = False
        return self.writer or None

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        obs = self.env.get_observations()
        privileged_obs = self.env.get_privileged_observations()
        critic_obs = privileged_obs if privileged_obs is not None else obs
        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
        self.alg.actor_critic.train()
        ep_infos = []
        rewbuffer = deque(maxlen=100)
        lenbuffer = deque(maxlen=100)
        cur_reward_sum = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        cur_episode_length = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        # Phase times on CUDA come from stream events read after update(), whose statistics readback
        # already waits for the stream: no extra host synchronisation between the rollout and the
        # update (upstream rsl_rl likewise times with time.time() and no sync).
        cuda = str(self.device).startswith("cuda")
        # Without a log directory nothing reads an iteration's statistics before the next one is
        # issued: the update is issued with a deferred readback and its statistics are taken once the
        # next rollout has been issued, so the GPU goes from the update straight into that rollout
        # (otherwise it idles ~0.3 ms per iteration while the host returns from the update's
        # synchronisation and issues again).  Same computation, same results.
        defer = cuda and self.log_dir is None
        pending = prev_end = None
        # act -> env.step -> process_env_step: each step's storage-row store rides on the next act's
        # launch (LGX_DEFER_STORE=0: its own launch, as before)
        self.alg.defer_store = os.environ.get("LGX_DEFER_STORE", "1") != "0"
        tot_iter = self.current_learning_iteration + num_learning_iterations
        completed = False
        try:
            for it in range(self.current_learning_iteration, tot_iter):
                start = time.time()
                if cuda:   # (the previous iteration's end event is this one's start: one marker less)
                    ev = [prev_end if prev_end is not None else torch.cuda.Event(enable_timing=True)] + \
                         [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    if prev_end is None:
                        ev[0].record()
                    prev_end = ev[2] if defer else None   # (synchronous runs: host logging lies between)
                with torch.inference_mode():
                    for _ in range(self.num_steps_per_env):
                        actions = self.alg.act(obs, critic_obs)
                        obs, privileged_obs, rewards, dones, infos = self.env.step(actions)
                        critic_obs = privileged_obs if privileged_obs is not None else obs
                        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
                        rewards, dones = rewards.to(self.device), dones.to(self.device)
                        self.alg.process_env_step(rewards, dones, infos)
                        if self.log_dir is not None:
                            if "episode" in infos:
                                ep_infos.append(infos["episode"])
                            cur_reward_sum += rewards
                            cur_episode_length += 1
                            new_ids = (dones > 0).nonzero(as_tuple=False)
                            rewbuffer.extend(cur_reward_sum[new_ids][:, 0].cpu().numpy().tolist())
                            lenbuffer.extend(cur_episode_length[new_ids][:, 0].cpu().numpy().tolist())
                            cur_reward_sum[new_ids] = 0
                            cur_episode_length[new_ids] = 0
                    if cuda:
                        ev[1].record()
                    stop = time.time()
                    collection_time = stop - start
                    start = stop
                    self.alg.flush_store()           # (the last step's storage row: no act follows it)
                    self.alg.compute_returns(critic_obs)
                if pending is not None:
                    p, pending = pending, None
                    self._finish_deferred(p)
                if defer:
                    self.alg.update(defer=True)
                    ev[2].record()
                    pending = ev
                    ep_infos.clear()
                    continue
                mean_value_loss, mean_surrogate_loss = self.alg.update()
                stop = time.time()
                learn_time = stop - start
                if cuda:
                    ev[2].record()
                    ev[2].synchronize()
                    collection_time = ev[0].elapsed_time(ev[1]) * 1e-3
                    learn_time = ev[1].elapsed_time(ev[2]) * 1e-3
                self.last_iteration_stats = dict(collection_time=collection_time, learn_time=learn_time,
                                                 value_loss=mean_value_loss, surrogate_loss=mean_surrogate_loss,
                                                 learning_rate=self.alg.learning_rate)
                if self.log_dir is not None:
                    self.log(locals())
                    if it % self.save_interval == 0:
                        self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
                ep_infos.clear()
            completed = True
        finally:
            # also on an exception: no deferred storage row may outlive learn() holding pointers to
            # the env's reward / reset / time-out buffers (the env has not stepped since that row's
            # process_env_step: every env.step follows an act, which takes the pending row), and no
            # update readback stays pending.  While an exception propagates (possibly a GPU error,
            # which the cleanup's launches and synchronisation would raise again) the cleanup is
            # best-effort and the original exception is the one reported.
            self.alg.defer_store = False
            p, pending = pending, None
            try:
                self.alg.flush_store()
                if p is not None:
                    self._finish_deferred(p)
            except Exception:
                if completed:
                    raise
                self.alg._pending_store = None
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))

    def _finish_deferred(self, ev):
        """Statistics of a deferred iteration: losses and learning rate from the update's readback,
        phase times from its stream events (all complete by the time the next rollout is issued)."""
        mean_value_loss, mean_surrogate_loss = self.alg.resolve()
        ev[2].synchronize()
        self.last_iteration_stats = dict(collection_time=ev[0].elapsed_time(ev[1]) * 1e-3,
                                         learn_time=ev[1].elapsed_time(ev[2]) * 1e-3,
                                         value_loss=mean_value_loss, surrogate_loss=mean_surrogate_loss,
                                         learning_rate=self.alg.learning_rate)

    def log(self, locs, width=80, pad=35):
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs
        self.tot_time += locs["collection_time"] + locs["learn_time"]
        it_time = locs["collection_time"] + locs["learn_time"]
        w = self._writer()
        lines = []
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                vals = torch.stack([torch.as_tensor(ep[key], device=self.device).reshape(()) for ep in locs["ep_infos"]])
                value = vals.mean().item()
                if w:
                    w.add_scalar("Episode/" + key, value, locs["it"])
                lines.append(f"{'Mean episode ' + key + ':':>{pad}} {value:.4f}")
        fps = int(self.num_steps_per_env * self.env.num_envs / it_time)
        if w:
            w.add_scalar("Loss/value_function", locs["mean_value_loss"], locs["it"])
            w.add_scalar("Loss/surrogate", locs["mean_surrogate_loss"], locs["it"])
            w.add_scalar("Loss/learning_rate", self.alg.learning_rate, locs["it"])
            w.add_scalar("Policy/mean_noise_std", self.alg.actor_critic.std.mean().item(), locs["it"])
            w.add_scalar("Perf/total_fps", fps, locs["it"])
            w.add_scalar("Perf/collection time", locs["collection_time"], locs["it"])
            w.add_scalar("Perf/learning_time", locs["learn_time"], locs["it"])
        header = f" \033[1m Learning iteration {locs['it']}/{self.current_learning_iteration + locs['num_learning_iterations']} \033[0m "
        s = f"{'#' * width}\n{header.center(width, ' ')}\n\n"
        s += f"{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, learning {locs['learn_time']:.3f}s)\n"
        s += f"{'Value function loss:':>{pad}} {locs['mean_value_loss']:.4f}\n"
        s += f"{'Surrogate loss:':>{pad}} {locs['mean_surrogate_loss']:.4f}\n"
        s += f"{'Mean action noise std:':>{pad}} {self.alg.actor_critic.std.mean().item():.2f}\n"
        if len(locs["rewbuffer"]) > 0:
            s += f"{'Mean reward:':>{pad}} {statistics.mean(locs['rewbuffer']):.2f}\n"
            s += f"{'Mean episode length:':>{pad}} {statistics.mean(locs['lenbuffer']):.2f}\n"
        s += "\n".join(lines) + "\n" + "-" * width + "\n"
        s += f"{'Total timesteps:':>{pad}} {self.tot_timesteps}\n{'Iteration time:':>{pad}} {it_time:.2f}s\n"
        print(s)

    def save(self, path, infos=None):
        torch.save({"model_state_dict": self.alg.actor_critic.state_dict(),
                    "optimizer_state_dict": self.alg.optimizer.state_dict(),
                    "iter": self.current_learning_iteration, "infos": infos}, path)

    def load(self, path, load_optimizer=True):
        d = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.actor_critic.load_state_dict(d["model_state_dict"])
        if hasattr(self.alg.actor_critic, "invalidate_fused"):
            self.alg.actor_critic.invalidate_fused()
        if load_optimizer:
            # as upstream rsl_rl: the optimizer state (its param_groups' lr included) is restored and
            # alg.learning_rate keeps the config value - the adaptive schedule's first update then
            # adapts from the config value and overwrites the restored lr, a fixed schedule steps
            # with the restored lr (tests/test_ppo.py::test_resume_learning_rate_follows_upstream)
            self.alg.optimizer.load_state_dict(d["optimizer_state_dict"])
        self.current_learning_iteration = d["iter"]
        return d["infos"]

    def get_inference_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_inference

    def close(self):
        """Release the update's collective resources (the lgx RCCL communicator of
        LGX_NATIVE_ALLREDUCE=1; collective: every rank calls it after its last learn())."""
        fused = getattr(self.alg, "_fused", None)
        if fused is not None:
            fused.close_comm()
