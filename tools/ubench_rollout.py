"""Rollout policy forward at N=4096 (actor+critic 235->512->256->128->{12,1}): the fused
lgx_mlp_forward_kernel vs the library path (batched GEMMs + lgx_bias_act) the PPO update uses."""
import torch

from legged_gym_amd.rl.actor_critic import ActorCritic


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
N = 4096
ac = ActorCritic(235, 235, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[512, 256, 128]).to(dev)
obs = torch.randn(N, 235, device=dev)
with torch.inference_mode():
    print("fused kernel us", t(lambda: ac.rollout_forward(obs, obs)))
    W1 = torch.cat([ac.actor[0].weight, ac.critic[0].weight]).t().contiguous()      # [235, 1024]
    W2 = torch.stack([ac.actor[2].weight.t(), ac.critic[2].weight.t()]).contiguous()  # [2,512,256]
    W3 = torch.stack([ac.actor[4].weight.t(), ac.critic[4].weight.t()]).contiguous()
    b1 = torch.cat([ac.actor[0].bias, ac.critic[0].bias])
    h1 = torch.empty(N, 1024, device=dev)
    h2 = torch.empty(2, N, 256, device=dev)
    h3 = torch.empty(2, N, 128, device=dev)

    def lib():
        torch.addmm(b1, obs, W1, out=h1)
        torch.nn.functional.elu(h1, inplace=True)
        x = h1.view(N, 2, 512).transpose(0, 1)
        torch.bmm(x, W2, out=h2)
        torch.nn.functional.elu(h2, inplace=True)
        torch.bmm(h2, W3, out=h3)
        torch.nn.functional.elu(h3, inplace=True)
    print("library path us", t(lib))
    print("  L1 addmm us", t(lambda: torch.addmm(b1, obs, W1, out=h1)))
    x = h1.view(N, 2, 512).transpose(0, 1)
    print("  L2 bmm us", t(lambda: torch.bmm(x, W2, out=h2)))
    print("  L3 bmm us", t(lambda: torch.bmm(h2, W3, out=h3)))
