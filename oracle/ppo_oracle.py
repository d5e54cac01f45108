"""ppo_oracle.py - CPU restatement (numpy, float64) of rsl_rl's PPO update.   TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, and only as the checker: never the product path (the
fused HIP update, rl/fused_ppo.py, or the autograd update in rl/ppo.py) and never a fallback.

What it restates: rsl_rl v1.0.x `PPO.update` (clipped surrogate, clipped value loss, entropy
bonus, adaptive-KL learning rate, `clip_grad_norm_`, `torch.optim.Adam`) and
`RolloutStorage.mini_batch_generator` (one `randperm` per update, the same permutation for every
epoch, transitions flattened time-major), for rsl_rl's `ActorCritic` (ELU MLPs, a state-independent
std parameter, `Normal(mean, std)` log-probabilities summed over actions).  Hyperparameters as
configured by legged_gym: `legged_robot_config.py:216-239` (LeggedRobotCfgPPO).  rsl_rl is an
external dependency that is absent from /root/reference and unpinned (`setup.py:11-13`,
SURVEY.md §8(c)): this restatement follows the published equations; parity against the
upstream package itself is UNPINNED.  Gradients are derived by hand (no autograd), so the
restatement is independent of torch and of the product's kernels.

Derivative rules of torch's elementwise max (`torch.max(a, b)`: the whole gradient to the
larger operand, half to each on a tie) and clamp (gradient 1 inside [lo, hi], bounds included).
Inside the clip range the two branches are equal up to rounding (tv + (v - tv) need not be v),
so which one a rounding-level difference selects does not change the derivative beyond rounding.
"""
import numpy as np

LOG_2PI = np.log(2.0 * np.pi)


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0.0)))


def elu_grad(x):
    return np.where(x > 0, 1.0, np.exp(np.minimum(x, 0.0)))


def mlp_forward(params, x):
    """params: [(W [out, in], b [out]), ...]; ELU after every layer but the last."""
    pre, acts = [], [x]
    h = x
    for i, (w, b) in enumerate(params):
        z = h @ w.T + b
        pre.append(z)
        h = elu(z) if i < len(params) - 1 else z
        acts.append(h)
    return h, pre, acts


def mlp_backward(params, pre, acts, g_out):
    grads = [None] * len(params)
    g = g_out
    for i in reversed(range(len(params))):
        w, _ = params[i]
        if i < len(params) - 1:
            g = g * elu_grad(pre[i])
        grads[i] = (g.T @ acts[i], g.sum(0))
        g = g @ w
    return grads


class Adam:
    """torch.optim.Adam defaults (betas 0.9 / 0.999, eps 1e-8, no weight decay)."""

    def __init__(self, shapes, b1=0.9, b2=0.999, eps=1e-8):
        self.m = [np.zeros(s) for s in shapes]
        self.v = [np.zeros(s) for s in shapes]
        self.t = 0
        self.b1, self.b2, self.eps = b1, b2, eps

    def step(self, params, grads, lr):
        self.t += 1
        bc1 = 1.0 - self.b1 ** self.t
        bc2 = 1.0 - self.b2 ** self.t
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            self.m[i] = self.b1 * self.m[i] + (1.0 - self.b1) * g
            self.v[i] = self.b2 * self.v[i] + (1.0 - self.b2) * g * g
            denom = np.sqrt(self.v[i]) / np.sqrt(bc2) + self.eps
            out.append(p - (lr / bc1) * self.m[i] / denom)
        return out


def _max_weights(a, b):
    """torch.max(a, b) backward: weight of the gradient that reaches a (b gets 1 - w)."""
    return np.where(a > b, 1.0, np.where(a == b, 0.5, 0.0))


def minibatch_grads(actor, critic, std, batch, idx, clip_param=0.2, value_loss_coef=1.0, entropy_coef=0.01,
                    use_clipped_value_loss=True):
    """Loss terms and d loss / d parameters of one minibatch (rows idx), before clipping:
    (value_loss, surrogate_loss, kl_mean, grads in the order actor (W, b)..., critic (W, b)...,
    std)."""
    mb = idx.shape[0]
    obs, cobs, act = batch["obs"][idx], batch["cobs"][idx], batch["actions"][idx]
    tv, adv, ret = batch["values"][idx, 0], batch["advantages"][idx, 0], batch["returns"][idx, 0]
    old_logp, old_mu, old_sigma = batch["logp"][idx, 0], batch["mu"][idx], batch["sigma"][idx]
    mu, pre_a, acts_a = mlp_forward(actor, obs)
    v, pre_c, acts_c = mlp_forward(critic, cobs)
    v = v[:, 0]
    sigma = np.broadcast_to(std, mu.shape)
    d = act - mu
    logp = np.sum(-d * d / (2.0 * sigma * sigma) - np.log(sigma) - 0.5 * LOG_2PI, axis=-1)
    kl = np.sum(np.log(sigma / old_sigma + 1.e-5) + (old_sigma ** 2 + (old_mu - mu) ** 2) / (2.0 * sigma ** 2) - 0.5,
                axis=-1)
    ratio = np.exp(logp - old_logp)
    s1 = -adv * ratio
    s2 = -adv * np.clip(ratio, 1.0 - clip_param, 1.0 + clip_param)
    surrogate_loss = np.maximum(s1, s2).mean()
    if use_clipped_value_loss:
        v_clip = tv + np.clip(v - tv, -clip_param, clip_param)
        l1, l2 = (v - ret) ** 2, (v_clip - ret) ** 2
        value_loss = np.maximum(l1, l2).mean()
        w = _max_weights(l1, l2)
        inside = np.abs(v - tv) <= clip_param
        g_v = (w * 2.0 * (v - ret) + (1.0 - w) * 2.0 * (v_clip - ret) * inside) / mb
    else:
        value_loss = ((ret - v) ** 2).mean()
        g_v = 2.0 * (v - ret) / mb
    g_v = value_loss_coef * g_v
    # d surrogate / d logp (through the ratio)
    w = _max_weights(s1, s2)
    inside = (ratio >= 1.0 - clip_param) & (ratio <= 1.0 + clip_param)
    g_logp = (w * -adv + (1.0 - w) * -adv * inside) / mb * ratio
    g_mu = g_logp[:, None] * d / (sigma * sigma)
    g_std = np.sum(g_logp[:, None] * (d * d / sigma ** 3 - 1.0 / sigma), axis=0)
    g_std = g_std - entropy_coef * (1.0 / std)          # - c_e * mean over rows of the entropy
    ga = mlp_backward(actor, pre_a, acts_a, g_mu)
    gc = mlp_backward(critic, pre_c, acts_c, g_v[:, None])
    grads = [a for wb in ga for a in wb] + [a for wb in gc for a in wb] + [g_std]
    return value_loss, surrogate_loss, kl.mean(), grads


def ppo_update(actor, critic, std, batch, perm, num_epochs, num_mini_batches, lr, clip_param=0.2,
               value_loss_coef=1.0, entropy_coef=0.01, max_grad_norm=1.0, desired_kl=0.01,
               schedule="adaptive", use_clipped_value_loss=True):
    """One PPO.update.

    actor / critic: [(W, b), ...] float64; std [A]; batch: dict of flattened transitions
    (obs, cobs, actions, values, advantages, returns, logp, mu, sigma; rows = T * N, time-major);
    perm: the update's permutation (torch.randperm's draw).  Returns (actor, critic, std, lr,
    mean_value_loss, mean_surrogate_loss, lr_per_minibatch)."""
    n_rows = perm.shape[0]
    mb = n_rows // num_mini_batches
    la = len(actor)
    params = [a for wb in actor for a in wb] + [a for wb in critic for a in wb] + [std]
    opt = Adam([p.shape for p in params])
    mean_v = mean_s = 0.0
    lrs = []

    def unpack(ps):
        a = [(ps[2 * i], ps[2 * i + 1]) for i in range(la)]
        c = [(ps[2 * la + 2 * i], ps[2 * la + 2 * i + 1]) for i in range(len(critic))]
        return a, c, ps[-1]

    for _ in range(num_epochs):
        for i in range(num_mini_batches):
            actor, critic, std = unpack(params)
            value_loss, surrogate_loss, kl_mean, grads = minibatch_grads(
                actor, critic, std, batch, perm[i * mb:(i + 1) * mb], clip_param, value_loss_coef, entropy_coef,
                use_clipped_value_loss)
            if desired_kl is not None and schedule == "adaptive":   # (under inference_mode: no gradient)
                if kl_mean > desired_kl * 2.0:
                    lr = max(1e-5, lr / 1.5)
                elif desired_kl / 2.0 > kl_mean > 0.0:
                    lr = min(1e-2, lr * 1.5)
            lrs.append(lr)
            total = np.sqrt(sum(float(np.sum(g * g)) for g in grads))
            coef = min(max_grad_norm / (total + 1e-6), 1.0)
            params = opt.step(params, [g * coef for g in grads], lr)
            mean_v += value_loss
            mean_s += surrogate_loss
    actor, critic, std = unpack(params)
    n = num_epochs * num_mini_batches
    return actor, critic, std, lr, mean_v / n, mean_s / n, lrs
