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
    # the same net on lgx_mlp_x3_forward (split-bf16, weights streamed from L2)
    from legged_gym_amd.sim import abi
    dims = (30, 128, 128, 128, 3)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    wl, bl = [], []
    for i in range(4):
        wi = torch.randn(dims[i + 1], dims[i], device=dev) / dims[i] ** 0.5
        t = torch.empty(int(lib.lgx_mlp_x3_weight_elems(dims[i + 1], dims[i])), dtype=torch.int16, device=dev)
        lgxlib.check(lib.lgx_mlp_x3_split(C.c_void_p(wi.data_ptr()), dims[i + 1], dims[i], C.c_void_p(t.data_ptr()),
                                          stream), "split")
        wl.append(t)
        bl.append(torch.randn(dims[i + 1], device=dev))
    d = (abi.LgxMlpX3Desc * 1)()
    d[0].x, d[0].y, d[0].rows, d[0].nl, d[0].act = x.data_ptr(), y.data_ptr(), rows, 4, 2
    for i, v in enumerate(dims):
        d[0].dims[i] = v
    for i in range(4):
        d[0].weights[i], d[0].biases[i] = wl[i].data_ptr(), bl[i].data_ptr()
    ms = timeit(lambda: lib.lgx_mlp_x3_forward(d, 1, stream))
    print(f"actuator-shaped mlp_x3 rows={rows}: {ms*1e3:.1f} us  {flop/ms/1e9:.1f} TFLOP/s")
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


def env_env_ab(task=os.environ.get("KB_TASK", "go1_rough"), n=int(os.environ.get("KB_N", "4096")),
               var=os.environ.get("KB_VAR", "LGX_ACT_FIRST"), modes=tuple(os.environ.get("KB_VALUES", "0,1").split(",")),
               rounds=int(os.environ.get("KB_ROUNDS", "10")), steps=24):
    """A/B of a per-launch env-step switch (env var `var`), interleaved in ONE process: every round
    times `steps` env steps per value (HIP events); prints median / min us per step."""
    from oracle_backend import make_env
    env = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
    env.reset()
    a = torch.randn(n, 12, device="cuda:0")
    res = {m: [] for m in modes}
    for r in range(rounds + 1):
        for m in modes:
            os.environ[var] = m
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                env.step(a)
            e1.record()
            e1.synchronize()
            if r:
                res[m].append(e0.elapsed_time(e1) * 1e3 / steps)
    for m in modes:
        v = sorted(res[m])
        print(f"{task} N={n} {var}={m}: env.step median {v[len(v) // 2]:.1f} us, min {v[0]:.1f} us", flush=True)


def env_create_ab(task=os.environ.get("KB_TASK", "go1_rough"), n=int(os.environ.get("KB_N", "4096")),
                  var=os.environ.get("KB_VAR", "LGX_ACT_OVERLAP"), modes=tuple(os.environ.get("KB_VALUES", "2,3").split(",")),
                  rounds=int(os.environ.get("KB_ROUNDS", "10")), steps=24):
    """A/B of an env switch read when the sim is created (env var `var`): one env per value, env
    steps interleaved round by round in ONE process (HIP events); prints median / min us per step."""
    from oracle_backend import make_env
    envs = {}
    prev = os.environ.get(var)
    for m in modes:
        os.environ[var] = m
        envs[m] = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
        envs[m].reset()
    if prev is None:
        os.environ.pop(var)
    else:
        os.environ[var] = prev
    a = torch.randn(n, 12, device="cuda:0")
    res = {m: [] for m in modes}
    for r in range(rounds + 1):
        for m in modes:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                envs[m].step(a)
            e1.record()
            e1.synchronize()
            if r:
                res[m].append(e0.elapsed_time(e1) * 1e3 / steps)
    for m in modes:
        v = sorted(res[m])
        print(f"{task} N={n} {var}={m}: env.step median {v[len(v) // 2]:.1f} us, min {v[0]:.1f} us", flush=True)


def phys_ab():
    """A/B the physics kernel lanes-per-leg variants (LGX_PHYS_PP, read when a sim is created)."""
    from oracle_backend import make_env
    for task in ("go1_flat_bench", "go1_rough"):
        envs = {}
        for pp in ("2", "4", "8"):
            os.environ["LGX_PHYS_PP"] = pp
            envs[pp] = make_env(task, num_envs=4096, device="cuda:0", backend="lgx")
            envs[pp].reset()
        os.environ.pop("LGX_PHYS_PP")
        for pp in ("2", "4", "8", "4", "8"):
            ms = timeit(lambda: envs[pp].simulate(4), iters=20)
            print(f"{task} physics 4 substeps N=4096 PP={pp}: {ms*1e3:.1f} us")


def ppo_ab(T=24, N=4096, OBS=235, ACT=12, modes=("lib", "auto", "lgx", "lib", "auto", "lgx"), gemms=True):
    """A/B the PPO update: hand-written fused GEMMs (lgx_gemm_nt) vs library GEMMs + epilogue
    passes, one full update (5 epochs x 4 minibatches) at the bench shape; plus per-GEMM timings."""
    import ctypes as C
    from legged_gym_amd.rl.actor_critic import ActorCritic
    from legged_gym_amd.rl.ppo import PPO
    from legged_gym_amd.sim import abi
    dev = "cuda:0"
    res = {}
    for mode in modes:
        os.environ["LGX_PPO_GEMM"] = mode
        torch.manual_seed(0)
        ac = ActorCritic(OBS, OBS, ACT, [512, 256, 128], [512, 256, 128]).to(dev)
        ppo = PPO(ac, num_learning_epochs=5, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95,
                  value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0,
                  schedule="adaptive", desired_kl=0.01, device=dev, use_fused_update=True)
        ppo.init_storage(N, T, [OBS], [None], [ACT])
        st = ppo.storage
        g = torch.Generator(device=dev).manual_seed(3)
        st.observations.copy_(torch.randn(T, N, OBS, device=dev, generator=g))
        st.actions.copy_(torch.randn(T, N, ACT, device=dev, generator=g))
        st.rewards.copy_(torch.randn(T, N, 1, device=dev, generator=g))
        st.values.copy_(torch.randn(T, N, 1, device=dev, generator=g))
        st.actions_log_prob.copy_(torch.randn(T, N, 1, device=dev, generator=g) * 0.3 - 17)
        st.mu.copy_(torch.randn(T, N, ACT, device=dev, generator=g) * 0.1)
        st.sigma.copy_(torch.rand(T, N, ACT, device=dev, generator=g) * 0.5 + 0.75)
        st.step = T
        st.compute_returns(torch.randn(N, 1, device=dev, generator=g), 0.99, 0.95)
        assert ppo._fused.lgx_gemm == (mode != "lib")
        ms = timeit(lambda: ppo.update(), iters=5, warm=2)
        res.setdefault(mode, []).append(ms)
        print(f"PPO update ({mode} GEMMs): {ms:.2f} ms", flush=True)
    os.environ.pop("LGX_PPO_GEMM")
    if gemms:
        gemm_bench(T * N // 4, torch_too=True)


def update_env_ab(var=os.environ.get("KB_VAR", "LGX_PPO_EARLY_REDUCE"), rounds=int(os.environ.get("KB_ROUNDS", "12")),
                  T=24, N=4096, OBS=235, ACT=12, modes=tuple(os.environ.get("KB_VALUES", "1,0").split(","))):
    """A/B of an update switch that is read per call / per minibatch (env var `var`, values `modes`),
    interleaved in ONE process on one PPO object: every round times one full update per value (HIP
    events), so box drift cancels (separate processes on one box drifted by +-5 %); prints median /
    min per value."""
    from legged_gym_amd.rl.actor_critic import ActorCritic
    from legged_gym_amd.rl.ppo import PPO
    dev = "cuda:0"
    torch.manual_seed(0)
    ac = ActorCritic(OBS, OBS, ACT, [512, 256, 128], [512, 256, 128]).to(dev)
    ppo = PPO(ac, num_learning_epochs=5, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95,
              value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0,
              schedule="adaptive", desired_kl=0.01, device=dev, use_fused_update=True)
    ppo.init_storage(N, T, [OBS], [None], [ACT])
    st = ppo.storage
    g = torch.Generator(device=dev).manual_seed(3)
    data = dict(observations=torch.randn(T, N, OBS, device=dev, generator=g),
                actions=torch.randn(T, N, ACT, device=dev, generator=g),
                rewards=torch.randn(T, N, 1, device=dev, generator=g),
                values=torch.randn(T, N, 1, device=dev, generator=g),
                actions_log_prob=torch.randn(T, N, 1, device=dev, generator=g) * 0.3 - 17,
                mu=torch.randn(T, N, ACT, device=dev, generator=g) * 0.1,
                sigma=torch.rand(T, N, ACT, device=dev, generator=g) * 0.5 + 0.75)
    last = torch.randn(N, 1, device=dev, generator=g)

    def one():
        for k, v in data.items():
            getattr(st, k).copy_(v)
        st.step = T
        st.compute_returns(last, 0.99, 0.95)
        ppo.update()
    res = {m: [] for m in modes}
    for r in range(rounds + 1):
        for m in modes:
            os.environ[var] = m
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            one()
            e1.record()
            e1.synchronize()
            if r:
                res[m].append(e0.elapsed_time(e1))
    for m in modes:
        v = sorted(res[m])
        print(f"{var}={m}: median {v[len(v) // 2]:.3f} ms, min {v[0]:.3f} ms over {len(v)} updates", flush=True)


def update_plan_ab(var=os.environ.get("KB_VAR", "LGX_PPO_TN_COLSUM"), rounds=int(os.environ.get("KB_ROUNDS", "12")),
                   T=24, N=4096, OBS=235, ACT=12,
                   modes=tuple(os.environ.get("KB_VALUES", "1,0").split(";" if ";" in os.environ.get("KB_VALUES", "")
                                                                          else ","))):
    """A/B of an update switch read when the update's launch plan is built (FusedPPOUpdate._alloc):
    one PPO object per value (built with `var` set, same seed and data), updates interleaved in ONE
    process (HIP events around each full update); prints median / min per value and the kernel
    time of one minibatch's backward is left to the rocprof trace."""
    from legged_gym_amd.rl.actor_critic import ActorCritic
    from legged_gym_amd.rl.ppo import PPO
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(3)
    data = dict(observations=torch.randn(T, N, OBS, device=dev, generator=g),
                actions=torch.randn(T, N, ACT, device=dev, generator=g),
                rewards=torch.randn(T, N, 1, device=dev, generator=g),
                values=torch.randn(T, N, 1, device=dev, generator=g),
                actions_log_prob=torch.randn(T, N, 1, device=dev, generator=g) * 0.3 - 17,
                mu=torch.randn(T, N, ACT, device=dev, generator=g) * 0.1,
                sigma=torch.rand(T, N, ACT, device=dev, generator=g) * 0.5 + 0.75)
    last = torch.randn(N, 1, device=dev, generator=g)
    ppos = {}

    def one(ppo):
        st = ppo.storage
        for k, v in data.items():
            getattr(st, k).copy_(v)
        st.step = T
        st.compute_returns(last, 0.99, 0.95)
        ppo.update()
    prev = os.environ.get(var)
    for m in modes:
        os.environ[var] = m
        torch.manual_seed(0)
        ac = ActorCritic(OBS, OBS, ACT, [512, 256, 128], [512, 256, 128]).to(dev)
        ppo = PPO(ac, num_learning_epochs=5, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95,
                  value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0,
                  schedule="adaptive", desired_kl=0.01, device=dev, use_fused_update=True)
        ppo.init_storage(N, T, [OBS], [None], [ACT])
        one(ppo)   # (builds the plan with `var` set)
        ppos[m] = ppo
    if prev is None:
        os.environ.pop(var)
    else:
        os.environ[var] = prev
    res = {m: [] for m in modes}
    for r in range(rounds):
        for m in modes:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            one(ppos[m])
            e1.record()
            e1.synchronize()
            res[m].append(e0.elapsed_time(e1))
    for m in modes:
        v = sorted(res[m])
        print(f"{var}={m}: median {v[len(v) // 2]:.3f} ms, min {v[0]:.3f} ms over {len(v)} updates", flush=True)


def gemm_bench(M=24576, torch_too=False, iters=20):
    """lgx_gemm_nt at the PPO-update shapes (and torch bmm without epilogue for reference)."""
    import ctypes as C
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim import lib as lgxlib
    dev = "cuda:0"
    lib = lgxlib.load()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    shapes = ((512, 256, 1), (256, 512, 1), (128, 256, 1), (256, 128, 3), (512, 256, 3))   # forwards, dA3, dA2
    if os.environ.get("KB_SHAPES"):   # "n,k,epi;n,k,epi..."
        shapes = [tuple(int(v) for v in s.split(",")) for s in os.environ["KB_SHAPES"].split(";")]
    for (n_, k_, epi) in shapes:
        A = torch.randn(2, M, k_, device=dev)
        B = torch.randn(2, n_, k_, device=dev)
        Cc = torch.empty(2, M, n_, device=dev)
        Y = torch.randn(2, M, n_, device=dev)
        bias = torch.randn(2, n_, device=dev)
        parts = torch.empty(lib.lgx_gemm_partials_floats(M, n_, 2), device=dev)
        a = abi.LgxGemmArgs()
        a.M, a.N, a.K, a.batch, a.epi = M, n_, k_, 2, epi
        a.A, a.lda, a.sa, a.B, a.ldb, a.sb = A.data_ptr(), k_, M * k_, B.data_ptr(), k_, n_ * k_
        a.C, a.ldc, a.sc, a.bias, a.Y, a.partials = Cc.data_ptr(), n_, M * n_, bias.data_ptr(), Y.data_ptr(), parts.data_ptr()
        f = 2.0 * 2 * M * n_ * k_
        algos = [int(x) for x in os.environ.get("KB_ALGOS", "1,2,3").split(",")]
        ld = lib.lgx_split_bf16_elems(1, k_)
        Bs = torch.zeros(2 * n_ * ld, dtype=torch.int16, device=dev)
        j = abi.LgxCopy2dJob()
        j.src, j.dst, j.src_ld, j.src_bs, j.dst_ld, j.dst_bs = B.data_ptr(), Bs.data_ptr(), k_, n_ * k_, ld, n_ * ld
        j.rows, j.cols, j.batch, j.transpose = n_, k_, 2, 0
        lgxlib.check(lib.lgx_split_bf16((abi.LgxCopy2dJob * 1)(j), 1, stream), "split")
        for algo in algos:   # 3 = split-bf16 with pre-split B
            a.algo = min(algo, 2)
            a.Bs = Bs.data_ptr() if algo == 3 else None
            t1 = timeit(lambda: lib.lgx_gemm_nt(C.byref(a), stream), iters=iters)
            if os.environ.get("KB_CLOCK"):   # X3P_CLOCK build: per-slot stamps of workgroup 0
                parts.zero_()
                lgxlib.check(lib.lgx_gemm_nt(C.byref(a), stream), "gemm")
                torch.cuda.synchronize()
                st = parts.view(torch.int64)[:8 * 32 * 8].view(8, 32, 8).double().cpu()
                valid = (st[:, :, 5] > 0) & (st[:, :, 0] > 0)
                for w in range(8):
                    v = valid[w]
                    d = st[w][v]
                    seg = [(d[:, e + 1] - d[:, e]).mean().item() for e in range(5)]
                    tot = (d[1:, 0] - d[:-1, 0]).mean().item() if v.sum() > 1 else 0
                    print(f"  wave {w}: slots {int(v.sum())} per-slot cycles {tot:.0f}: wait {seg[0]:.0f} "
                          f"barrier {seg[1]:.0f} issue {seg[2]:.0f} stores {seg[3]:.0f} compute {seg[4]:.0f}", flush=True)
            print(f"gemm M={M} N={n_} K={k_} epi={epi} algo={algo}: lgx {t1*1e3:.1f} us "
                  f"{f/t1/1e9:.1f} TF/s", flush=True)
        if torch_too:
            t2 = timeit(lambda: torch.bmm(A, B.transpose(1, 2), out=Cc), iters=iters)
            print(f"  torch bmm (no epilogue) {t2*1e3:.1f} us {f/t2/1e9:.1f} TF/s", flush=True)


def tn_bench(M=24576, iters=20):
    """lgx_gemm_tn (dW GEMMs) at the PPO-update shapes vs torch bmm over row slices."""
    import ctypes as C
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim import lib as lgxlib
    dev = "cuda:0"
    lib = lgxlib.load()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for (R, Cc, ldb) in ((512, 235, 256), (256, 512, 512), (128, 256, 256)):
        A = torch.randn(2, M, R, device=dev)
        B = torch.randn(2, M, ldb, device=dev)
        f = 2.0 * 2 * M * R * Cc
        for S in [int(x) for x in os.environ.get("KB_SLICES", "8,16,32").split(",")]:
            Cbuf = torch.empty(2 * S * R * Cc + 1024, device=dev)   # (+ a tail for TN_CLOCK stamps)
            Cout = Cbuf[:2 * S * R * Cc].view(2, S, R, Cc)
            a = abi.LgxGemmTnArgs()
            a.M, a.R, a.Cc, a.slices, a.batch = M, R, Cc, S, 2
            a.A, a.lda, a.sa, a.B, a.ldb, a.sb = A.data_ptr(), R, M * R, B.data_ptr(), ldb, M * ldb
            a.C, a.ldc = Cout.data_ptr(), Cc
            t1 = timeit(lambda: lgxlib.check(lib.lgx_gemm_tn(C.byref(a), stream), "tn"), iters=iters)
            if os.environ.get("KB_CLOCK"):   # TN_CLOCK build: per-stage stamps of workgroup 0's first tile
                Cbuf.zero_()
                lgxlib.check(lib.lgx_gemm_tn(C.byref(a), stream), "tn")
                torch.cuda.synchronize()
                st = Cbuf[2 * S * R * Cc:].view(torch.int64)[:4 * 32 * 4].view(4, 32, 4).double().cpu()
                for w in range(4):   # (8-wave kernel: rows 0, 1 = waves 0 and 4)
                    d = st[w][(st[w, :, 3] > 0) & (st[w, :, 0] > 0)]
                    if len(d) < 2:
                        continue
                    per = (d[1:, 0] - d[:-1, 0]).mean().item()
                    seg = [(d[:, e + 1] - d[:, e]).mean().item() for e in range(3)]
                    print(f"  wave {w}: stages {len(d)} per-stage {per:.0f}: compute {seg[0]:.0f} split+write {seg[1]:.0f} "
                          f"load-issue {seg[2]:.0f} barrier {per - sum(seg):.0f}", flush=True)
            if os.environ.get("KB_WSCLOCK"):   # TN_WS_CLOCK build: consumer start/end, producer start/end per stage
                Cbuf.zero_()
                lgxlib.check(lib.lgx_gemm_tn(C.byref(a), stream), "tn")
                torch.cuda.synchronize()
                st = Cbuf[2 * S * R * Cc:].view(torch.int64)[:32 * 4].view(32, 4).double().cpu()
                v = st[(st > 0).all(1)]
                if len(v) > 2:
                    per = (v[1:, 0] - v[:-1, 0]).mean().item()
                    print(f"  per-stage {per:.0f}: consumer compute {(v[:, 1] - v[:, 0]).mean().item():.0f}, "
                          f"producer write {(v[:, 3] - v[:, 2]).mean().item():.0f}, producer start - consumer start "
                          f"{(v[:, 2] - v[:, 0]).mean().item():.0f}", flush=True)
            P = torch.empty(2 * S, R, Cc, device=dev)
            Bv = B[..., :Cc].reshape(2 * S, M // S, Cc) if ldb == Cc else B.view(2 * S, M // S, ldb)[..., :Cc]
            t2 = timeit(lambda: torch.bmm(A.view(2 * S, M // S, R).transpose(1, 2), Bv, out=P), iters=iters)
            print(f"gemm_tn R={R} Cc={Cc} S={S}: lgx {t1*1e3:.1f} us {f/t1/1e9:.1f} TF/s; torch bmm {t2*1e3:.1f} us "
                  f"{f/t2/1e9:.1f} TF/s", flush=True)


def phys_run(task="go1_rough", n=4096, steps=int(os.environ.get("KB_STEPS", "10"))):
    """Short env-step loop for PMC collection (rocprofv3 --pmc): 10 env steps after reset."""
    from oracle_backend import make_env
    env = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(steps):
        env.step(torch.randn(n, 12, device="cuda:0", generator=g) * 0.5)
    torch.cuda.synchronize()
    from legged_gym_amd.sim import lib as lgxlib
    L = lgxlib.load()
    if hasattr(L, "lgx_debug_clock"):   # LGX_PHASE_CLOCK_BUF build: per-workgroup clocks of the last launch
        import ctypes as C
        import numpy as np
        nb = (n + 15) // 16
        buf = np.zeros((nb, 14), dtype=np.uint64)
        L.lgx_debug_clock(buf.ctypes.data_as(C.c_void_p), C.c_int32(nb))
        os.makedirs("gpurun_out", exist_ok=True)
        np.save(os.environ.get("KB_CLK_OUT", "gpurun_out/clk.npy"), buf)


if __name__ == "__main__":
    what = sys.argv[1:] or ["mlp", "env"]
    if "mlp" in what:
        mlp_bench()
    if "env" in what:
        env_bench()
    if "phys" in what:
        phys_ab()
    if "physrun" in what:
        phys_run()
    if "ppo" in what:
        ppo_ab()
    for m in ("lib", "auto", "lgx"):
        if f"ppo_{m}" in what:
            ppo_ab(modes=(m,), gemms=False)
    if "gemm" in what:
        gemm_bench(M=int(os.environ.get("KB_M", "24576")), torch_too="torch" in what)
    if "tn" in what:
        tn_bench()
    if "update_env" in what:
        update_env_ab()
    if "update_plan" in what:
        update_plan_ab()
    if "env_env" in what:
        env_env_ab()
    if "env_create" in what:
        env_create_ab()


