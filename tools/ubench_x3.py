"""Rollout policy forward on lgx_mlp_x3_kernel (actor + critic 235->512->256->128->{12,1}, one
launch): time per launch at 4096 / 8192 rows.  With LGX_LIB_PATH=tools/_tmp/clock/liblgx.so
(tools/phase_clock.sh) the kernel also prints wave 0's phase cycles of workgroup 0 per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from legged_gym_amd.rl.actor_critic import ActorCritic  # noqa: E402


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
clock = "clock" in os.environ.get("LGX_LIB_PATH", "")
ac = ActorCritic(235, 235, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[512, 256, 128]).to(dev)
with torch.inference_mode():
    for N in (4096, 8192):
        obs = torch.randn(N, 235, device=dev)
        ref = (ac.actor(obs), ac.critic(obs))
        m, v = ac.rollout_forward(obs, obs)
        err = max((m - ref[0]).abs().max().item(), (v - ref[1]).abs().max().item())
        us = t(lambda: ac.rollout_forward(obs, obs), it=3 if clock else 50)
        print(f"N={N} x3 actor+critic {us:7.1f} us  max|err| vs torch {err:.2e}", flush=True)
