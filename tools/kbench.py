"""Kernel micro-benchmarks on the GPU box (timing with torch.cuda events on the launch stream)."""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def mlp_bench():
    from legged_gym_amd.envs.go1.go1 import pack_uninet_weights
    from legged_gym_amd.rl.actor_critic import ActorCritic
    from legged_gym_amd.sim import lib as lgxlib
    from legged_gym_amd.sim.model import load_actuator_net
    import legged_gym_amd
    dev = torch.device("cuda:0")
    lib = lgxlib.load()
    net = load_actuator_net(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources/actuator_nets/go1_net.npz"))
    w = torch.tensor(pack_uninet_weights(net), device=dev)
    sc = torch.tensor(net["vel_std"], device=dev)
    rows = 4 * 4096 * 4
    x = torch.randn(rows, 30, device=dev)
    y = torch.empty(rows, 3, device=dev)
    fn = lambda: lib.lgx_actuator_mlp(C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), rows, C.c_void_p(w.data_ptr()),
                                      C.c_void_p(sc.data_ptr()), None)
    ms = timeit(fn)
    flop = rows * 2 * (30 * 128 + 128 * 128 * 2 + 128 * 3)
    print(f"actuator mlp rows={rows}: {ms*1e3:.1f} us  {flop/ms/1e9:.1f} TFLOP/s")
    ac = ActorCritic(235, 235, 12, [512, 256, 128], [512, 256, 128]).to(dev)
    obs = torch.randn(4096, 235, device=dev)
    with torch.inference_mode():
        ms = timeit(lambda: ac.act_and_evaluate(obs, obs))
        flop = 4096 * 2 * 2 * (235 * 512 + 512 * 256 + 256 * 128 + 128 * 6.5)
        print(f"actor+critic act_and_evaluate rows=4096: {ms*1e3:.1f} us  {flop/ms/1e9:.1f} TFLOP/s")
        ms2 = timeit(lambda: (ac.actor(obs), ac.critic(obs)))
        print(f"  torch (hipBLASLt) actor+critic: {ms2*1e3:.1f} us")
        big = torch.randn(24576, 235, device=dev)
        ms3 = timeit(lambda: ac._fused_actor(big), iters=20)
        f3 = 24576 * 2 * (235 * 512 + 512 * 256 + 256 * 128 + 128 * 12)
        print(f"actor fused rows=24576: {ms3*1e3:.1f} us {f3/ms3/1e9:.1f} TFLOP/s; torch {timeit(lambda: ac.actor(big), iters=20)*1e3:.1f} us")


def env_bench(task="go1_rough", n=4096):
    from oracle_backend import make_env
    env = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
    env.reset()
    a = torch.randn(n, 12, device="cuda:0") * 0.5
    ms = timeit(lambda: env.step(a), iters=50)
    print(f"{task} env.step N={n}: {ms*1e3:.1f} us/step  {n/ms*1e3/1e6:.2f} M env-steps/s (env only)")


def phys_ab():
    """A/B the physics kernel lanes-per-leg variants in one process."""
    import ctypes as C
    from oracle_backend import make_env
    for task in ("go1_flat_bench", "go1_rough"):
        env = make_env(task, num_envs=4096, device="cuda:0", backend="lgx")
        env.reset()
        for pp in ("2", "4", "8", "4", "8"):
            os.environ["LGX_PHYS_PP"] = pp
            ms = timeit(lambda: env.simulate(4), iters=20)
            print(f"{task} physics 4 substeps N=4096 PP={pp}: {ms*1e3:.1f} us")
        os.environ.pop("LGX_PHYS_PP")


def mlp_ab():
    """A/B the wide (policy) MLP tile height: rollout actor+critic on 4096 rows."""
    from legged_gym_amd.rl.actor_critic import ActorCritic
    ac = ActorCritic(235, 235, 12, [512, 256, 128], [512, 256, 128]).cuda()
    x = torch.randn(4096, 235, device="cuda:0")
    f = 2 * 4096 * 2 * (235 * 512 + 512 * 256 + 256 * 128 + 128 * 6.5)
    with torch.inference_mode():
        ref = (ac.actor(x), ac.critic(x))
        for rs in ("1", "1"):
            os.environ["LGX_MLP_WIDE_RS"] = rs
            m, v = ac.rollout_forward(x, x)
            err = max((m - ref[0]).abs().max().item(), (v - ref[1]).abs().max().item())
            ms = timeit(lambda: ac.rollout_forward(x, x), iters=50)
            print(f"rollout MLP RS={rs}: {ms*1e3:.1f} us {f/ms/1e9:.1f} TFLOP/s  max|err| {err:.2e}")
    os.environ.pop("LGX_MLP_WIDE_RS")


def phys_run(task="go1_rough", n=4096, steps=10):
    """Short env-step loop for PMC collection (rocprofv3 --pmc): 10 env steps after reset."""
    from oracle_backend import make_env
    env = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(steps):
        env.step(torch.randn(n, 12, device="cuda:0", generator=g) * 0.5)
    torch.cuda.synchronize()


if __name__ == "__main__":
    what = sys.argv[1:] or ["mlp", "env"]
    if "mlp" in what:
        mlp_bench()
    if "env" in what:
        env_bench()
    if "phys" in what:
        phys_ab()
    if "mlpab" in what:
        mlp_ab()
    if "physrun" in what:
        phys_run()


