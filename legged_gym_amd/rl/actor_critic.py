"""rsl_rl-compatible ActorCritic (the policy the reference trains: legged_robot_config.py:216-224,
built by OnPolicyRunner at task_registry.py:160; upstream rsl_rl v1.0.x `ActorCritic`).

Training forward/backward uses torch autograd (library GEMMs).  The no-grad rollout forward
(`act` under inference mode, `act_inference`, `evaluate`) runs on the lgx fused MLP kernel
(f32 MFMA, all layers in one launch with the activations resident in LDS) when the module
lives on a GPU; weights are re-transposed for the kernel lazily after each optimizer step.
"""
import ctypes as C

import torch
import torch.nn as nn
from torch.distributions import Normal


def get_activation(name):
    table = {"elu": nn.ELU(), "selu": nn.SELU(), "relu": nn.ReLU(), "crelu": nn.ReLU(), "lrelu": nn.LeakyReLU(),
             "tanh": nn.Tanh(), "sigmoid": nn.Sigmoid()}
    if name not in table:
        print("invalid activation function!")
        return None
    return table[name]


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is computed as S batched partial products summed
    over S (split-K over the PPO minibatch dimension).  The library's single GEMM for
    dW = dY^T X at M = 24576 rows launches only (out/32 x in/256) tiles and runs at ~20 TFLOP/s;
    S = 8 partial GEMMs fill the 256 CUs (2-5x faster on MI355X, tools/ubench.py)."""

    @staticmethod
    def forward(ctx, x, w, b, splits):
        ctx.save_for_backward(x, w)
        ctx.splits = splits
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        S = ctx.splits
        gx = gy @ w if ctx.needs_input_grad[0] else None
        M, N = gy.shape
        K = x.shape[1]
        gw = torch.bmm(gy.reshape(S, M // S, N).transpose(1, 2), x.reshape(S, M // S, K)).sum(0)
        gb = gy.sum(0)
        return gx, gw, gb, None


class LgxLinear(nn.Linear):
    """nn.Linear (same parameters / state_dict) with the split-K weight gradient on GPU."""

    def forward(self, x):
        if x.is_cuda and torch.is_grad_enabled() and x.dim() == 2 and x.shape[0] >= 4096:
            for s in (8, 4, 2):
                if x.shape[0] % s == 0:
                    return _SplitKLinearFn.apply(x, self.weight, self.bias, s)
        return super().forward(x)


def _mlp(n_in, hidden, n_out, act):
    layers = [LgxLinear(n_in, hidden[0]), act]
    for i in range(len(hidden)):
        if i == len(hidden) - 1:
            layers.append(LgxLinear(hidden[i], n_out))
        else:
            layers += [LgxLinear(hidden[i], hidden[i + 1]), act]
    return nn.Sequential(*layers)


class _FusedMLP:
    """Inference-only view of an nn.Sequential(Linear, act, ..., Linear) on the fused MLP kernels:
    lgx_mlp_x3_forward (split-bf16 MFMA products, weights pre-split once per parameter version)
    by default, lgx_mlp_forward_batch (f32 MFMA) with LGX_MLP_X3=0 or when the activations of
    32 rows do not fit the LDS."""

    ACT = {nn.ELU: 1, nn.Tanh: 2}

    def __init__(self, seq):
        import os
        self.linears = [m for m in seq if isinstance(m, nn.Linear)]
        acts = {type(m) for m in seq if not isinstance(m, nn.Linear)}
        self.act = self.ACT.get(next(iter(acts)), 0) if len(acts) == 1 else 0
        self.dims = [self.linears[0].in_features] + [l.out_features for l in self.linears]
        self.ok = self.act != 0 and max(self.dims) <= 512 and len(self.linears) <= 6
        self.x3 = self.ok and os.environ.get("LGX_MLP_X3", "1") != "0"   # split-bf16 kernel allowed
        self.last_x3 = None          # which kernel the last launch with this network ran (tests)
        self._ver = {}               # parameter version each weight image was built from
        self._wt = self._b = self._wl = None

    def _refresh(self, x3):
        """Biases and the weight image of the requested kernel, rebuilt when the parameters changed
        (optimizer step, load) - split-bf16 limb images for lgx_mlp_x3_forward, transposed f32
        weights for lgx_mlp_forward_batch; a network may launch with either, per launch."""
        ver = tuple(l.weight._version for l in self.linears) + tuple(l.bias._version for l in self.linears)
        dev = self.linears[0].weight.device
        n = len(self.linears)
        with torch.no_grad():
            if self._ver.get("b") != ver or self._b is None or self._b[0].device != dev:
                self._b = [l.bias.detach().contiguous() for l in self.linears]
                self._bp = (C.c_void_p * n)(*[t.data_ptr() for t in self._b])
                self._dims_c = (C.c_int32 * (n + 1))(*self.dims)
                self._ver["b"] = ver
            if x3 and (self._ver.get("wl") != ver or self._wl is None or self._wl[0].device != dev):
                from legged_gym_amd.sim import lib as lgxlib
                lib = lgxlib.load()
                stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                if self._wl is None or self._wl[0].device != dev:
                    self._wl = [torch.empty(int(lib.lgx_mlp_x3_weight_elems(l.out_features, l.in_features)),
                                            dtype=torch.int16, device=dev) for l in self.linears]
                ws = [l.weight.detach().contiguous() for l in self.linears]   # (views of the flat buffer)
                wp = (C.c_void_p * n)(*[w.data_ptr() for w in ws])
                dp = (C.c_void_p * n)(*[wl.data_ptr() for wl in self._wl])
                dims = (C.c_int32 * (n + 1))(*self.dims)
                lgxlib.check(lib.lgx_mlp_x3_split_layers(wp, dims, n, dp, stream), "lgx_mlp_x3_split")   # one launch
                self._split_keep = ws
                self._ver["wl"] = ver
            if not x3 and (self._ver.get("wt") != ver or self._wt is None or self._wt[0].device != dev):
                self._wt = [l.weight.detach().t().contiguous() for l in self.linears]
                self._wp = (C.c_void_p * n)(*[t.data_ptr() for t in self._wt])
                self._ver["wt"] = ver

    def desc(self, x, y, x3=None):
        from legged_gym_amd.sim import abi
        x3 = self.x3 if x3 is None else x3
        self._refresh(x3)
        self.last_x3 = x3
        if x3:
            d = abi.LgxMlpX3Desc()
            d.x, d.y, d.rows, d.nl, d.act = x.data_ptr(), y.data_ptr(), x.shape[0], len(self.linears), self.act
            for i, v in enumerate(self.dims):
                d.dims[i] = v
            for i in range(len(self.linears)):
                d.weights[i] = self._wl[i].data_ptr()
                d.biases[i] = self._b[i].data_ptr()
            return d
        d = abi.LgxMlpDesc()
        d.x, d.y, d.rows, d.nl, d.act = x.data_ptr(), y.data_ptr(), x.shape[0], len(self.linears), self.act
        for i, v in enumerate(self.dims):
            d.dims[i] = v
        for i in range(len(self.linears)):
            d.weights[i] = self._wt[i].data_ptr()
            d.biases[i] = self._b[i].data_ptr()
        return d

    def invalidate(self):
        self._ver = {}

    def __call__(self, x):
        return run_fused([(self, x)])[0]


def launch_forward(descs, count, stream):
    """`count` (1 or 2) MLP descriptors in one lgx_mlp_forward_batch / lgx_mlp_x3_forward launch
    on `stream` (by descriptor type)."""
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    if isinstance(descs[0], abi.LgxMlpX3Desc):
        lgxlib.check(lib.lgx_mlp_x3_forward(descs, count, stream), "lgx_mlp_x3_forward")
    else:
        lgxlib.check(lib.lgx_mlp_forward_batch(descs, count, stream), "lgx_mlp_forward_batch")


def _x3_fits(mlps):
    """One lgx_mlp_x3_forward launch holds these networks' activations in LDS (decided once per
    combination, from dims alone)."""
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim import lib as lgxlib
    key = tuple(tuple(m.dims) for m in mlps) + tuple(m.act for m in mlps)
    fit = _X3_FIT.get(key)
    if fit is None:
        ds = (abi.LgxMlpX3Desc * len(mlps))()
        for d, m in zip(ds, mlps):
            d.nl, d.act, d.rows = len(m.linears), m.act, 1
            for i, v in enumerate(m.dims):
                d.dims[i] = v
        fit = _X3_FIT[key] = lgxlib.load().lgx_mlp_x3_lds_bytes(ds, len(mlps)) >= 0
    return fit


_X3_FIT = {}


def make_descs(triples):
    """Descriptor array of one fused launch over up to two (fused_mlp, input, output) triples:
    split-bf16 (lgx_mlp_x3_forward) when every network takes it and their activations fit the LDS
    together, else f32 MFMA (lgx_mlp_forward_batch) for all of them.  Decided per launch: a pair
    that does not fit together leaves each network's own (single-network) launches on split-bf16."""
    from legged_gym_amd.sim import abi
    mlps = [m for m, _, _ in triples]
    x3 = all(m.x3 for m in mlps) and _x3_fits(mlps)
    descs = ((abi.LgxMlpX3Desc if x3 else abi.LgxMlpDesc) * len(triples))()
    for i, (m, x, y) in enumerate(triples):
        descs[i] = m.desc(x, y, x3)
    return descs


def run_fused(pairs):
    """Forward of up to two (fused_mlp, input) pairs in one launch."""
    triples = []
    for m, x in pairs:
        x = x.contiguous()
        triples.append((m, x, torch.empty(x.shape[0], m.dims[-1], device=x.device, dtype=torch.float)))
    launch_forward(make_descs(triples), len(triples),
                   C.c_void_p(torch.cuda.current_stream(pairs[0][1].device).cuda_stream))
    return [y for _, _, y in triples]


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=(256, 256, 256),
                 critic_hidden_dims=(256, 256, 256), activation="elu", init_noise_std=1.0, **kwargs):
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs.keys())))
        super().__init__()
        act = get_activation(activation)
        self.actor = _mlp(num_actor_obs, list(actor_hidden_dims), num_actions, act)
        self.critic = _mlp(num_critic_obs, list(critic_hidden_dims), 1, act)
        print(f"Actor MLP: {self.actor}")
        print(f"Critic MLP: {self.critic}")
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        Normal.set_default_validate_args(False)
        self._fused_actor = _FusedMLP(self.actor)
        self._fused_critic = _FusedMLP(self.critic)
        self.use_fused_inference = True

    @staticmethod
    def init_weights(sequential, scales):
        [torch.nn.init.orthogonal_(module.weight, gain=scales[idx]) for idx, module in
         enumerate(mod for mod in sequential if isinstance(mod, nn.Linear))]

    def reset(self, dones=None):
        pass

    def invalidate_fused(self):
        """Call after parameters change outside autograd-visible in-place ops (optimizer step, load)."""
        self._fused_actor.invalidate()
        self._fused_critic.invalidate()

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def _fused_ok(self, x, fused):
        return (self.use_fused_inference and fused.ok and x.is_cuda and
                (torch.is_inference_mode_enabled() or not torch.is_grad_enabled()))

    def _actor_mean(self, observations):
        if self._fused_ok(observations, self._fused_actor):
            return self._fused_actor(observations)
        return self.actor(observations)

    def update_distribution(self, observations):
        mean = self._actor_mean(observations)
        self.distribution = Normal(mean, mean * 0.0 + self.std)

    def act(self, observations, **kwargs):
        self.update_distribution(observations)
        return self.distribution.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_inference(self, observations):
        return self._actor_mean(observations)

    def act_and_evaluate(self, observations, critic_observations):
        """Rollout fast path: actor mean + critic value in ONE fused MFMA launch, then sample."""
        if self._fused_ok(observations, self._fused_actor) and self._fused_critic.ok:
            mean, value = run_fused([(self._fused_actor, observations), (self._fused_critic, critic_observations)])
            self.distribution = Normal(mean, mean * 0.0 + self.std)
            return self.distribution.sample(), value
        return self.act(observations), self.evaluate(critic_observations)

    def rollout_forward(self, observations, critic_observations):
        """(actor mean, critic value) in one fused MFMA launch, or None when the fused kernel does
        not apply (CPU, non-ELU/tanh stacks, widths > 512)."""
        if self._fused_ok(observations, self._fused_actor) and self._fused_critic.ok:
            mean, value = run_fused([(self._fused_actor, observations), (self._fused_critic, critic_observations)])
            return mean, value
        return None

    def evaluate(self, critic_observations, **kwargs):
        if self._fused_ok(critic_observations, self._fused_critic):
            return self._fused_critic(critic_observations)
        return self.critic(critic_observations)


# ---------------------------------------------------------------------------------------------
# Recurrent policy (rsl_rl v1.0.x `ActorCriticRecurrent` / `Memory`; legged_robot_config.py:221-224
# names its options rnn_type / rnn_hidden_size / rnn_num_layers).  The LSTM / GRU runs on torch
# (MIOpen); the MLP heads behind it keep the fused rollout kernels of ActorCritic.

def split_and_pad_trajectories(tensor, dones):
    """[T, N, ...] -> ([T, n_traj, ...] zero-padded trajectories, [T, n_traj] masks): the rollout cut
    at every done (and at the end), env-major (rsl_rl utils.split_and_pad_trajectories)."""
    dones = dones.clone()
    dones[-1] = 1
    flat_dones = dones.transpose(1, 0).reshape(-1, 1)
    done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64), flat_dones.nonzero()[:, 0]))
    lengths = done_indices[1:] - done_indices[:-1]
    trajectories = torch.split(tensor.transpose(1, 0).flatten(0, 1), lengths.tolist())
    # one full-length dummy so the padding always reaches T, removed afterwards
    trajectories = trajectories + (torch.zeros(tensor.shape[0], *tensor.shape[2:], device=tensor.device,
                                               dtype=tensor.dtype),)
    padded = torch.nn.utils.rnn.pad_sequence(trajectories)[:, :-1]
    masks = lengths > torch.arange(0, tensor.shape[0], device=tensor.device).unsqueeze(1)
    return padded, masks


def unpad_trajectories(trajectories, masks):
    """Inverse of split_and_pad_trajectories: [T, n_traj, H] -> [T, N, H]."""
    return trajectories.transpose(1, 0)[masks.transpose(1, 0)].view(
        -1, trajectories.shape[0], trajectories.shape[-1]).transpose(1, 0)


class Memory(nn.Module):
    """rsl_rl Memory: one LSTM (or GRU) over the observation stream.  Rollout (masks None): one time
    step from the stored hidden state; update (masks given): whole padded trajectories from the
    hidden states saved at their first step, unpadded back to [T, envs, H]."""

    def __init__(self, input_size, type="lstm", num_layers=1, hidden_size=256):
        super().__init__()
        rnn_cls = nn.GRU if type.lower() == "gru" else nn.LSTM
        self.rnn = rnn_cls(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers)
        self.hidden_states = None

    def forward(self, input, masks=None, hidden_states=None):
        if masks is not None:
            if hidden_states is None:
                raise ValueError("Hidden states not passed to memory module during policy update")
            out, _ = self.rnn(input, hidden_states)
            return unpad_trajectories(out, masks)
        out, self.hidden_states = self.rnn(input.unsqueeze(0), self.hidden_states)
        return out

    def reset(self, dones=None):
        if self.hidden_states is None:
            return
        # LSTM: (h, c); GRU: one tensor whose layers are iterated - both [.., envs, hidden]
        for hidden_state in self.hidden_states:
            hidden_state[..., dones, :] = 0.0


class ActorCriticRecurrent(ActorCritic):
    is_recurrent = True

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=(256, 256, 256),
                 critic_hidden_dims=(256, 256, 256), activation="elu", rnn_type="lstm", rnn_hidden_size=256,
                 rnn_num_layers=1, init_noise_std=1.0, **kwargs):
        if kwargs:
            print("ActorCriticRecurrent.__init__ got unexpected arguments, which will be ignored: "
                  + str(kwargs.keys()))
        super().__init__(num_actor_obs=rnn_hidden_size, num_critic_obs=rnn_hidden_size, num_actions=num_actions,
                         actor_hidden_dims=actor_hidden_dims, critic_hidden_dims=critic_hidden_dims,
                         activation=activation, init_noise_std=init_noise_std)
        self.memory_a = Memory(num_actor_obs, type=rnn_type, num_layers=rnn_num_layers, hidden_size=rnn_hidden_size)
        self.memory_c = Memory(num_critic_obs, type=rnn_type, num_layers=rnn_num_layers, hidden_size=rnn_hidden_size)
        print(f"Actor RNN: {self.memory_a}")
        print(f"Critic RNN: {self.memory_c}")

    def reset(self, dones=None):
        self.memory_a.reset(dones)
        self.memory_c.reset(dones)

    def act(self, observations, masks=None, hidden_states=None):
        input_a = self.memory_a(observations, masks, hidden_states)
        return super().act(input_a.squeeze(0))

    def act_inference(self, observations):
        input_a = self.memory_a(observations)
        return super().act_inference(input_a.squeeze(0))

    def evaluate(self, critic_observations, masks=None, hidden_states=None):
        input_c = self.memory_c(critic_observations, masks, hidden_states)
        return super().evaluate(input_c.squeeze(0))

    def act_and_evaluate(self, observations, critic_observations):
        """act + evaluate (both memories advance one step); the two MLP heads in one fused launch."""
        input_a = self.memory_a(observations).squeeze(0)
        input_c = self.memory_c(critic_observations).squeeze(0)
        if self._fused_ok(input_a, self._fused_actor) and self._fused_critic.ok:
            mean, value = run_fused([(self._fused_actor, input_a), (self._fused_critic, input_c)])
            self.distribution = Normal(mean, mean * 0.0 + self.std)
            return self.distribution.sample(), value
        return ActorCritic.act(self, input_a), ActorCritic.evaluate(self, input_c)

    # the fused rollout path of PPO._act_fused feeds observations straight into the actor MLP
    rollout_forward = None

    def get_hidden_states(self):
        return self.memory_a.hidden_states, self.memory_c.hidden_states
