"""Rollout policy forward (actor+critic 235->512->256->128->{12,1}): the single fused launch
(lgx_mlp_forward_batch, LGX_MLP_WAVES variants) vs one tiled launch per layer (layered)."""
import os

import torch

import legged_gym_amd.rl.actor_critic as acm
from legged_gym_amd.rl.actor_critic import ActorCritic, run_fused


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = "cuda"
ac = ActorCritic(235, 235, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[512, 256, 128]).to(dev)
flop_net = 2 * (235 * 512 + 512 * 256 + 256 * 128 + 128 * 6.5)
with torch.inference_mode():
    for N in (4096, 8192):
        obs = torch.randn(N, 235, device=dev)
        ref = (ac.actor(obs), ac.critic(obs))
        for name, rows, waves in (("fused w4", 0, "4"), ("fused w8", 0, "8"), ("fused 32x8", 0, "16"),
                                  ("layered", 1, "4")):
            acm.LAYERED_MIN_ROWS = rows
            os.environ["LGX_MLP_WAVES"] = waves
            m, v = ac.rollout_forward(obs, obs)
            err = max((m - ref[0]).abs().max().item(), (v - ref[1]).abs().max().item())
            us2 = t(lambda: ac.rollout_forward(obs, obs))
            us1 = t(lambda: run_fused([(ac._fused_actor, obs)]))
            print(f"N={N} {name:10s} actor+critic {us2:7.1f} us ({2 * N * flop_net / us2 / 1e6:5.1f} TF)  "
                  f"actor {us1:7.1f} us  max|err| {err:.2e}")
