"""Rollout storage with the rsl_rl RolloutStorage contract (transitions, GAE, minibatches).

GAE (rsl_rl compute_returns: gamma/lam recursion with done masking, then advantage
normalisation) runs as ONE HIP kernel (lgx GAE, one thread per env over the T steps) on the
GPU; in a data-parallel run the normalisation statistics are global: every rank's (count, mean,
M2) summaries of its advantages (float64) are gathered in rank order and combined with Chan's
pairwise formula, so N ranks x B envs normalise like 1 rank x N*B envs (no sum / sum-of-squares
cancellation when |mean| >> std).
"""
import math

import torch


def moments_combine(a, b):
    """Chan et al.'s pairwise combination of (count, mean, M2) summaries (lgx_rl.hip)."""
    n = a[0] + b[0]
    if n == 0.0:
        return a
    d = b[1] - a[1]
    return (n, a[1] + d * (b[0] / n), a[2] + b[2] + d * d * (a[0] * b[0] / n))


def local_moments(x):
    """(count, mean, M2) of x as a float64 [3] tensor (two passes)."""
    xd = x.double().reshape(-1)
    mean = xd.mean()
    return torch.stack([torch.tensor(float(xd.numel()), dtype=torch.float64, device=x.device), mean,
                        ((xd - mean) ** 2).sum()])


def combined_mean_std(parts):
    """(mean, unbiased std) as Python floats from a flat [3 k] tensor of summaries, combined in order."""
    s = (0.0, 0.0, 0.0)
    for n, m, m2 in parts.detach().double().cpu().view(-1, 3).tolist():
        s = moments_combine(s, (n, m, m2))
    var = s[2] / (s[0] - 1.0) if s[0] > 1.0 else 0.0
    return s[1], math.sqrt(var)


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.critic_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None
            self.in_storage = False   # row already written by the fused rollout kernel

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, actions_shape,
                 device="cpu"):
        self.device = device
        self.obs_shape = obs_shape
        self.privileged_obs_shape = privileged_obs_shape
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs
        f = dict(device=device)
        self.observations = torch.zeros(T, N, *obs_shape, **f)
        self.privileged_observations = (torch.zeros(T, N, *privileged_obs_shape, **f)
                                        if privileged_obs_shape[0] is not None else None)
        self.rewards = torch.zeros(T, N, 1, **f)
        self.actions = torch.zeros(T, N, *actions_shape, **f)
        self.dones = torch.zeros(T, N, 1, **f).byte()
        self.actions_log_prob = torch.zeros(T, N, 1, **f)
        self.values = torch.zeros(T, N, 1, **f)
        self.returns = torch.zeros(T, N, 1, **f)
        self.advantages = torch.zeros(T, N, 1, **f)
        self.mu = torch.zeros(T, N, *actions_shape, **f)
        self.sigma = torch.zeros(T, N, *actions_shape, **f)
        self.num_transitions_per_env = T
        self.num_envs = N
        self.step = 0
        self.saved_hidden_states_a = None   # recurrent policies: memory state before each step
        self.saved_hidden_states_c = None

    def add_transitions(self, t: "RolloutStorage.Transition"):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        s = self.step
        self.observations[s].copy_(t.observations)
        if self.privileged_observations is not None:
            self.privileged_observations[s].copy_(t.critic_observations)
        self.actions[s].copy_(t.actions)
        self.rewards[s].copy_(t.rewards.view(-1, 1))
        self.dones[s].copy_(t.dones.view(-1, 1))
        self.values[s].copy_(t.values)
        self.actions_log_prob[s].copy_(t.actions_log_prob.view(-1, 1))
        self.mu[s].copy_(t.action_mean)
        self.sigma[s].copy_(t.action_sigma)
        self._save_hidden_states(t.hidden_states)
        self.step += 1

    def _save_hidden_states(self, hidden_states):
        """rsl_rl RolloutStorage._save_hidden_states: [T, layers, envs, hidden] per state tensor
        (LSTM: h and c; GRU: one), zero until the memory has run once."""
        if hidden_states is None or hidden_states == (None, None):
            return
        hid_a = hidden_states[0] if isinstance(hidden_states[0], tuple) else (hidden_states[0],)
        hid_c = hidden_states[1] if isinstance(hidden_states[1], tuple) else (hidden_states[1],)
        if self.saved_hidden_states_a is None:
            T = self.observations.shape[0]
            self.saved_hidden_states_a = [torch.zeros(T, *h.shape, device=self.device) for h in hid_a]
            self.saved_hidden_states_c = [torch.zeros(T, *h.shape, device=self.device) for h in hid_c]
        for i in range(len(hid_a)):
            self.saved_hidden_states_a[i][self.step].copy_(hid_a[i])
            self.saved_hidden_states_c[i][self.step].copy_(hid_c[i])

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam, reduce_stats=None):
        """rsl_rl RolloutStorage.compute_returns.  reduce_stats (data-parallel): a callable taking this
        rank's flat float64 (count, mean, M2) summaries and returning every rank's, concatenated in
        rank order (PPO._gather_moments)."""
        if self.returns.is_cuda:
            from legged_gym_amd.rl import fused
            if reduce_stats is None:   # one process: the normalisation rides on the GAE launch pair
                fused.gae_norm(self.rewards, self.values, self.dones, last_values.contiguous(), self.returns,
                               self.advantages, gamma, lam)
                return
            # data-parallel: the same per-workgroup summaries, every rank's combined in rank order
            # (at world 1 bitwise lgx_gae_norm)
            parts = fused.gae_parts(self.rewards, self.values, self.dones, last_values.contiguous(), self.returns,
                                    self.advantages, gamma, lam)
            fused.adv_norm(self.advantages, reduce_stats(parts))
            return
        else:
            advantage = 0
            for step in reversed(range(self.num_transitions_per_env)):
                next_values = last_values if step == self.num_transitions_per_env - 1 else self.values[step + 1]
                not_term = 1.0 - self.dones[step].float()
                delta = self.rewards[step] + not_term * gamma * next_values - self.values[step]
                advantage = delta + not_term * gamma * lam * advantage
                self.returns[step] = advantage + self.values[step]
            self.advantages = self.returns - self.values
        adv = self.advantages
        if reduce_stats is None:
            mean, std = adv.mean(), adv.std()
            self.advantages = (adv - mean) / (std + 1e-8)
        else:   # f32 mean / std from the float64 global statistics, as lgx_adv_norm
            mean, std = combined_mean_std(reduce_stats(local_moments(adv)))
            self.advantages = (adv - torch.tensor(mean, dtype=adv.dtype)) / (
                torch.tensor(std, dtype=adv.dtype) + 1e-8)

    def get_statistics(self):
        done = self.dones.clone()
        done[-1] = 1
        flat = done.permute(1, 0, 2).reshape(-1, 1)
        idx = torch.cat((flat.new_tensor([-1], dtype=torch.int64), flat.nonzero(as_tuple=False)[:, 0]))
        lengths = idx[1:] - idx[:-1]
        return lengths.float().mean(), self.rewards.mean()

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        batch_size = self.num_envs * self.num_transitions_per_env
        mb = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mb, requires_grad=False, device=self.device)
        obs = self.observations.flatten(0, 1)
        cobs = self.privileged_observations.flatten(0, 1) if self.privileged_observations is not None else obs
        actions = self.actions.flatten(0, 1)
        values = self.values.flatten(0, 1)
        returns = self.returns.flatten(0, 1)
        old_logp = self.actions_log_prob.flatten(0, 1)
        adv = self.advantages.flatten(0, 1)
        mu = self.mu.flatten(0, 1)
        sigma = self.sigma.flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                b = indices[i * mb:(i + 1) * mb]
                yield obs[b], cobs[b], actions[b], values[b], adv[b], returns[b], old_logp[b], mu[b], sigma[b], \
                    (None, None), None

    def reccurent_mini_batch_generator(self, num_mini_batches, num_epochs=8):
        """rsl_rl RolloutStorage.reccurent_mini_batch_generator (upstream's spelling): minibatches of
        whole envs; observations as zero-padded trajectories with their masks, the memories' hidden
        states at each trajectory's first step.  As upstream v1.0.x, an LSTM's critic batch receives
        the ACTOR's saved states (`hid_c_batch = ... else hid_a_batch`), kept for parity."""
        from .actor_critic import split_and_pad_trajectories
        padded_obs, traj_masks = split_and_pad_trajectories(self.observations, self.dones)
        if self.privileged_observations is not None:
            padded_cobs, _ = split_and_pad_trajectories(self.privileged_observations, self.dones)
        else:
            padded_cobs = padded_obs
        mb = self.num_envs // num_mini_batches
        for _ in range(num_epochs):
            first_traj = 0
            for i in range(num_mini_batches):
                start, stop = i * mb, (i + 1) * mb
                dones = self.dones.squeeze(-1)
                last_was_done = torch.zeros_like(dones, dtype=torch.bool)
                last_was_done[1:] = dones[:-1]
                last_was_done[0] = True
                last_traj = first_traj + int(torch.sum(last_was_done[:, start:stop]))
                masks_b = traj_masks[:, first_traj:last_traj]
                obs_b = padded_obs[:, first_traj:last_traj]
                cobs_b = padded_cobs[:, first_traj:last_traj]
                lwd = last_was_done.permute(1, 0)
                hid_a = [h.permute(2, 0, 1, 3)[lwd][first_traj:last_traj].transpose(1, 0).contiguous()
                         for h in self.saved_hidden_states_a]
                hid_c = [h.permute(2, 0, 1, 3)[lwd][first_traj:last_traj].transpose(1, 0).contiguous()
                         for h in self.saved_hidden_states_c]
                hid_a = hid_a[0] if len(hid_a) == 1 else hid_a
                hid_c = hid_c[0] if len(hid_c) == 1 else hid_a
                yield (obs_b, cobs_b, self.actions[:, start:stop], self.values[:, start:stop],
                       self.advantages[:, start:stop], self.returns[:, start:stop],
                       self.actions_log_prob[:, start:stop], self.mu[:, start:stop], self.sigma[:, start:stop],
                       (hid_a, hid_c), masks_b)
                first_traj = last_traj
