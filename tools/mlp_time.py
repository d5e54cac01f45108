"""Time the rollout actor + critic forward (one lgx_mlp_x3_forward launch, 4096 rows; MT_N) for
each variant library named on the command line: `product` = the in-tree liblgx.so, any other name =
tools/_tmp/v_<name>/liblgx.so (built with tools/ab_build.sh and copied there). DESIGN.md §4.4."""
import os, subprocess, sys
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    import torch
    sys.path.insert(0, os.getcwd())
    from legged_gym_amd.rl.actor_critic import ActorCritic
    dev = "cuda:0"
    torch.manual_seed(0)
    ac = ActorCritic(235, 235, 12, [512, 256, 128], [512, 256, 128]).to(dev)
    obs = torch.randn(int(os.environ.get("MT_N", "4096")), 235, device=dev)
    res = []
    with torch.inference_mode():
        mu0 = ac.rollout_forward(obs, obs)
        for rep in range(5):
            for _ in range(20): ac.rollout_forward(obs, obs)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(200): ac.rollout_forward(obs, obs)
            e.record(); torch.cuda.synchronize()
            res.append(s.elapsed_time(e) / 200 * 1e3)
    ref = ac.actor(obs)
    print("max |mu - torch| =", float((mu0[0] - ref).abs().max()), "checksum", repr(float(mu0[0].double().sum())),
          repr(float(mu0[1].double().sum())))
    print(f"{os.environ.get('LGX_LIB_PATH','product')}: per call {min(res):.1f} us (min of 5), {sorted(res)[2]:.1f} median")
    sys.exit(0)
for v in sys.argv[1:]:
    env = dict(os.environ, LGX_LIB_PATH=os.path.abspath(f"tools/_tmp/v_{v}/liblgx.so") if v != "product" else "")
    if v == "product": env.pop("LGX_LIB_PATH")
    r = subprocess.run([sys.executable, __file__, "--one"], env=env, timeout=300)
    if r.returncode: sys.exit(r.returncode)
