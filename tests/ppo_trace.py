"""Test helper: record every optimizer step of a fused PPO update (FusedPPOUpdate) - the flat
parameters, Adam moments and step counter before it, the minibatch rows, the flat gradient the
step consumed (after the data-parallel all-reduce, before clipping), the learning rate it used and
the parameters after it - so that tests can check EVERY coordinate of EVERY step:
  * the gradient against an independent evaluation (autograd / the numpy oracle) at the recorded
    parameters and rows,
  * the step against float64 torch Adam + clip_grad_norm_ applied to that gradient.
"""
import numpy as np
import torch


class _LibSpy:
    """Forwards every attribute to the product library; the Adam entry points first snapshot the
    flat gradient they are about to consume (stream-ordered clone: after the backward and the
    data-parallel all-reduce, before the step clips it in place as clip_grad_norm_ does)."""

    def __init__(self, lib, fused, sink):
        self._lib, self._fused, self._sink = lib, fused, sink

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if name not in ("lgx_adam_clip", "lgx_adam_clip_mirror", "lgx_adam_clip_mirror_sq"):
            return fn

        def wrapped(*args):
            # (the _sq entry takes the reductions' sums of squares and no grad_scale: 1)
            grad_scale = 1.0 if name.endswith("_sq") else float(args[7].value if hasattr(args[7], "value") else args[7])
            self._sink.append((self._fused.flat_g.clone(), grad_scale))
            return fn(*args)
        return wrapped


class StepTrace:
    def __init__(self, fused):
        self.fused = fused
        self.steps = []
        self._orig = fused._minibatch_body
        self._orig_lib = fused.lib
        self._grads = []
        fused.lib = _LibSpy(fused.lib, fused, self._grads)

        def body(idx, obs, cobs, args, stream, apply=True, xs=None):
            f = self.fused
            if not apply:
                return self._orig(idx, obs, cobs, args, stream, apply, xs)
            o = f.optimizer
            rec = dict(idx=idx.clone(), p0=f.flat_p.clone(), m0=o.m.clone(), v0=o.v.clone(),
                       step0=int(o.step_dev.item()))
            n0 = len(self._grads)
            self._orig(idx, obs, cobs, args, stream, apply, xs)
            assert len(self._grads) == n0 + 1, "one optimizer step per minibatch"
            g_raw, grad_scale = self._grads[-1]
            # the gradient of the step: the (all-reduced) sum x grad_scale = the rank average
            rec.update(g=g_raw * grad_scale, g_clipped=f.flat_g.clone(), lr=float(o.lr_dev.item()),
                       p1=f.flat_p.clone(), m1=o.m.clone(), v1=o.v.clone())
            self.steps.append(rec)
        fused._minibatch_body = body

    def close(self):
        self.fused._minibatch_body = self._orig
        self.fused.lib = self._orig_lib


def adam64(rec, max_norm, betas=(0.9, 0.999), eps=1e-8):
    """float64 torch.optim.Adam (no weight decay) after clip_grad_norm_(max_norm) on the recorded
    gradient: (p1, m1, v1) expected."""
    g = rec["g"].double()
    norm = g.norm().item()
    coef = min(max_norm / (norm + 1e-6), 1.0) if max_norm > 0 else 1.0
    g = g * coef      # (the step leaves this clipped gradient in the flat gradient buffer)
    b1, b2 = betas
    t = rec["step0"] + 1
    m = b1 * rec["m0"].double() + (1 - b1) * g
    v = b2 * rec["v0"].double() + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
    denom = v.sqrt() / np.sqrt(bc2) + eps
    p = rec["p0"].double() - (rec["lr"] / bc1) * m / denom
    return p, m, v


def flat_view(fused, tensors):
    """A flat vector in the fused layout from per-parameter tensors (ActorCritic.parameters() order)."""
    out = torch.zeros(fused.n, dtype=torch.float64, device=fused.flat_p.device)
    for p, t in zip(fused.optimizer.params, tensors):
        off = fused.off[id(p)]
        out[off:off + p.numel()] = t.reshape(-1).to(out)
    return out
