"""bench.py — headline measurement: rsl_rl-style PPO training throughput (env-steps/s, whole
node) for Go1 on rough trimesh terrain with the 187-point height scan, 4096 envs per GPU
(BASELINE.json metric; workload = configs[2] "C3", which fits one GPU; N>1 = configs[3]).

One "step" = one PPO iteration: 24 x (policy act on the fused MFMA MLP + lgx_step) + GAE +
5 epochs x 4 minibatches of PPO (fused f32-MFMA update, RCCL gradient all-reduce when N>1).
value = 24 * envs_per_gpu * world * K / max-over-ranks wall time of K iterations.

Launch: python bench.py [--gpus N --steps K --warmup W].  Under torch.distributed.run (one rank
per GPU, env vars RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) WORLD_SIZE must equal --gpus; without a
launcher, --gpus N > 1 starts the N ranks itself (torch.distributed.run as a child process, before
anything touches the GPU), passes rank 0's JSON line through and exits with the launcher's code.
"""
import argparse
import ctypes as C
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic work per env-step: physics kernel = fused 4 substeps (VALU),
# actuator MLP = 4 substeps x 4 legs x 2 x (30*128 + 128*128*2 + 128*3) FLOP
ACT_MLP_FLOP_PER_ENV_STEP = 4 * 4 * 2 * (30 * 128 + 128 * 128 * 2 + 128 * 3)
MI355X_F32_PEAK_TFLOPS = 157.3      # vector FP32 == f32 MFMA peak (MI355X_MICROARCH.md)
MI355X_HBM_PEAK_GBS = 8000.0
# PMC figures (rocprofv3 --pmc passes of the same build, tools/gpu_profile.sh): HBM bytes per launch
# = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads) and MFMA utilisation.
# Default: the newest committed profiles/r*_pmc_{env,ppo}_kernels.json; LGX_BENCH_PMC_ENV /
# LGX_BENCH_PMC_PPO point at a fresh pair from the same GPU session.  A file is used only for the
# workload it was collected on (its "workload" entry; files without one are go1_rough, 4096 envs).
import glob  # noqa: E402


def _newest(kind):
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{kind}_kernels.json")))
    return files[-1] if files else ""


PMC_FILE = os.environ.get("LGX_BENCH_PMC_ENV") or _newest("env")
PPO_PMC_FILE = os.environ.get("LGX_BENCH_PMC_PPO") or _newest("ppo")
MI355X_BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA (MI355X_MICROARCH.md)
SPLIT_PRODUCTS = 6                  # split-bf16: six bf16 limb products per f32 product (lgx_gemm_split.hip)
MI355X_SIMDS = 256 * 4              # MfmaUtil's SIMD_NUM (counter_defs.yaml): 256 CUs x 4 SIMDs
MI355X_XCDS = 8                     # GRBM_GUI_ACTIVE arrives summed over the 8 XCDs


def _pmc_passes(path, task, n_envs):
    """The passes of a PMC summary file if it was collected on (task, n_envs), else None."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    wl = d.get("workload", {"task": "go1_rough", "num_envs": 4096})
    return d.get("passes") if (wl.get("task"), int(wl.get("num_envs", 0))) == (task, n_envs) else None


def pmc_traffic_bytes(kernel, task, n_envs, fetch_pass="fetch", write_pass="write"):
    p = _pmc_passes(PMC_FILE, task, n_envs)
    try:
        return int((2 * p[fetch_pass][kernel]["FETCH_SIZE"] + p[write_pass][kernel]["WRITE_SIZE"]) * 1024)
    except (TypeError, KeyError):
        return None


def gemm_kernel_info(key, split):
    """(kernel name pattern as rocprof reports it, compute pipe, peak in f32-product TFLOP/s) of the
    PPO GEMM launches timed under `key` (an lgx_gemm_nt epilogue, or "tn" = lgx_gemm_tn)."""
    pipe = "bf16 MFMA (v_mfma_f32_32x32x16_bf16), split-bf16: 6 limb products per f32 product"
    if key == "tn":
        return "gemm_tn_*_kernel<*>", pipe, MI355X_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
    if split:   # the pipelined kernel (lgx_gemm_x3p.hip)
        return f"gemm_nt_x3p_kernel<{key}, *>", pipe, MI355X_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
    return f"gemm_nt_kernel<8, {key}>", "f32 MFMA (v_mfma_f32_32x32x2_f32)", MI355X_F32_PEAK_TFLOPS
GEMM_NOTES = {1: "lgx_gemm_nt LGX_GEMM_BIAS_ELU: hidden-layer forwards of actor and critic (235->512 with K padded "
                 "to 256, 512->256, 256->128)",
              2: "lgx_gemm_nt LGX_GEMM_DELU_COLSUM: backward dA of the hidden layers (512x256 and 256x128 weights)",
              3: "lgx_gemm_nt LGX_GEMM_DELU: backward dA of the hidden layers (512x256 and 256x128 weights; the "
                 "bias gradients come from lgx_gemm_tn's column sums)",
              "tn": "lgx_gemm_tn: weight gradients dW_k = dZ_k^T Y_{k-1} of the hidden layers over row slices "
                    "(512x235, 256x512 on the LDS-ring gemm_tn_ring_kernel<256>; 128x256 on gemm_tn_ring_kernel<128>; "
                    "per network)"}


# the MFMA kernels of one iteration whose utilisation the bench line reports (PMC pass "mfma")
MFMA_KERNELS = ["gemm_tn_*_kernel<*>", "gemm_nt_x3p_kernel<1, *>", "gemm_nt_x3p_kernel<3, *>", "lgx_mlp_x3_kernel*",
                "lgx_post_physics_act_kernel*"]


def _ppo_matches(p, kernel, passname):
    import fnmatch
    return [(name, v) for name, v in p.get(passname, {}).items() if fnmatch.fnmatchcase(name, kernel)]


def pmc_ppo_traffic_bytes(kernel, task, n_envs):
    """HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KB) of a PPO-update kernel from the PMC
    passes over one bench iteration of (task, n_envs); `kernel` may hold '*' wildcards (e.g. the
    K-specialised instantiations of one epilogue): dispatch-weighted mean over the matches."""
    p = _pmc_passes(PPO_PMC_FILE, task, n_envs)
    if not p:
        return None
    tot = n = 0.0
    for name, f in _ppo_matches(p, kernel, "fetch"):
        w = p.get("write", {}).get(name)
        if w is None or "FETCH_SIZE" not in f or "WRITE_SIZE" not in w:
            continue
        d = f.get("dispatches", 1)
        tot += d * (2 * f["FETCH_SIZE"] + w["WRITE_SIZE"]) * 1024
        n += d
    return int(tot / n) if n else None


def pmc_mfma_busy(kernel, task, n_envs):
    """MFMA utilisation of the kernels matching `kernel` in the PMC pass "mfma" of (task, n_envs):
    SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) / (SIMDs x kernel cycles), kernel cycles =
    GRBM_GUI_ACTIVE / XCDs (rocprofv3's MfmaUtil), summed over the dispatches of every match; None
    when the file has no such pass.  rocprofv3 serialises dispatches under --pmc, so second-stream
    kernels are measured alone there."""
    p = _pmc_passes(PPO_PMC_FILE, task, n_envs)
    if not p:
        return None
    busy = cyc = insts = disp = 0.0
    for _, c in _ppo_matches(p, kernel, "mfma"):
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or not c.get("GRBM_GUI_ACTIVE"):
            continue
        d = c.get("dispatches", 1)
        busy += d * c["SQ_VALU_MFMA_BUSY_CYCLES"]
        cyc += d * c["GRBM_GUI_ACTIVE"] / MI355X_XCDS
        insts += d * c.get("SQ_INSTS_MFMA", 0.0)
        disp += d
    if not cyc:
        return None
    return {"mfma_busy": busy / (MI355X_SIMDS * cyc), "mfma_insts_per_launch": insts / disp,
            "kernel_cycles_per_launch": cyc / disp, "dispatches": int(disp),
            "source": os.path.relpath(PPO_PMC_FILE, ROOT) + " pass mfma"}


from legged_gym_amd.sim.flops import physics_flop_per_env_substep, policy_flop_per_sample  # noqa: E402

# compulsory HBM bytes per env-step outside the PPO storage: physics state
# in/out + actuator-net rows, post-physics gathers/obs/heights/state
ENV_BYTES_PER_ENV_STEP = (3.0e6 + 11.9e6) / 4096 + 3.7e3


def iteration_roofline(runner, env, N, it_ms):
    """T_roof = sum over phases of max(bytes / HBM peak, FLOP / compute peak) for
    one PPO iteration on one GPU; frac = T_roof / measured iteration time."""
    alg, ac, st = runner.alg, runner.alg.actor_critic, runner.alg.storage
    dims = lambda seq: [m.in_features for m in seq if hasattr(m, "in_features")][:1] + \
        [m.out_features for m in seq if hasattr(m, "out_features")]
    fwd, epoch = policy_flop_per_sample(dims(ac.actor), dims(ac.critic))
    samples = runner.num_steps_per_env * N
    row_bytes = sum(t[0].numel() * t.element_size() for t in (
        st.observations, st.actions, st.rewards, st.dones, st.values, st.returns, st.advantages,
        st.actions_log_prob, st.mu, st.sigma)) / st.num_envs   # storage row bytes per sample
    decim = env.cfg.control.decimation
    # f32-accurate MFMA work is priced at the split-bf16 rate (bf16 dense peak / 6 limb products:
    # 417 TF/s of f32 products, above the 157 TF/s f32 MFMA), the physics at the FP32 VALU peak
    split_peak = MI355X_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
    phases = {
        "physics (fp32 VALU)": (samples * decim * physics_flop_per_env_substep(
            env._lgx_model.num_points, 4.0, env.cfg.terrain.mesh_type in ("heightfield", "trimesh")),
            samples * ENV_BYTES_PER_ENV_STEP, MI355X_F32_PEAK_TFLOPS),
        "actuator net (f32-accurate MFMA)": (samples * ACT_MLP_FLOP_PER_ENV_STEP if hasattr(env, "_actuator_dvel")
                                             else 0, 0, split_peak),
        "rollout policy forward (f32-accurate MFMA)": (samples * fwd, 0, split_peak),
        "PPO update (f32-accurate MFMA)": (alg.num_learning_epochs * samples * epoch,
                                           samples * row_bytes * (1 + alg.num_learning_epochs), split_peak),
    }
    out, t_roof = {}, 0.0
    for name, (flop, nbytes, peak) in phases.items():
        t = max(flop / (peak * 1e12), nbytes / (MI355X_HBM_PEAK_GBS * 1e9)) * 1e3
        out[name] = {"flop": flop, "hbm_bytes": int(nbytes), "t_roof_ms": round(t, 4)}
        t_roof += t
    return {"t_roof_ms": round(t_roof, 3), "t_measured_ms": round(it_ms, 3), "frac": t_roof / it_ms,
            "peaks": {"f32_tflops": MI355X_F32_PEAK_TFLOPS, "split_bf16_f32_product_tflops": split_peak,
                      "hbm_gbs": MI355X_HBM_PEAK_GBS}, "phases": out}


BASELINE_METRIC = "env-steps/sec (whole node), Go1 rough-terrain 4096 envs/GPU at 1/2/4/8 GPUs"
WORKLOADS = {
    "go1_rough": "C3 go1_rough: Go1 trimesh curriculum terrain + 187-point height scan, actuator-net history+MLP",
    "go1_flat_bench": "C2 go1_flat_bench: Go1 flat, PD drive, no domain randomisation",
    "anymal_c_rough": "C5 anymal_c_rough: ANYmal-C trimesh curriculum terrain + 187-point height scan, friction/mass "
                      "randomisation, pushes",
    "cassie": "cassie: the biped (2 legs x 6 joints, dense joint-space physics kernel) on trimesh curriculum terrain "
              "+ 121-point height scan",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--task", default="go1_rough")
    p.add_argument("--num_envs", type=int, default=4096)
    p.add_argument("--no_cpu_baseline", action="store_true")
    p.add_argument("--cpu_envs", type=int, default=4096)
    p.add_argument("--actuator_net_torques", action="store_true",
                   help="ANYmal: the SEA actuator network as the torque source (cfg.control.explicit_torques)")
    p.add_argument("--rendezvous_only", action="store_true",
                   help="launch contract check without a GPU: every rank joins a gloo group, the ranks are counted "
                        "with an all-reduce, rank 0 prints them; LGX_BENCH_FAIL_RANK=r makes rank r exit with code 3 "
                        "after the count (tests/test_bench_cli.py: the launcher's exit code carries one rank's failure)")
    return p.parse_args()


def mlp_flop_per_sample(dims):
    return 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))


def _host_cpu_info():
    """lscpu-style facts of the host the CPU baseline runs on (model, sockets, physical cores,
    hardware threads) plus the CPUs this process may use (affinity, cgroup quota)."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        phys, model = set(), ""
        with open("/proc/cpuinfo") as f:
            pid = cid = None
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and not model:
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    cid = v
                elif not k and pid is not None:
                    phys.add((pid, cid))
                    pid = cid = None
        info.update(cpu_model=model, sockets=len({p for p, _ in phys}) or None, physical_cores=len(phys) or None)
    except OSError:
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpu_quota"] = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    return info


def _cpu_iteration(task, n_envs, steps_per_env, threads):
    """Env-steps/s of one PPO iteration (collection + learn) of the C oracle env (OpenMP over envs)
    + torch-CPU ActorCritic/PPO at `threads` threads, after one untimed warm-up iteration."""
    import torch
    from oracle_backend import make_env, load_oracle
    from legged_gym_amd.rl.runner import OnPolicyRunner
    from legged_gym_amd.utils.helpers import class_to_dict
    from legged_gym_amd.utils.task_registry import task_registry
    torch.set_num_threads(threads)
    load_oracle().lgxo_set_threads(C.c_int(threads))   # the oracle's OpenMP env loops
    env = make_env(task, num_envs=n_envs, device="cpu", backend="oracle")
    _, train_cfg = task_registry.get_cfgs(task)
    tc = class_to_dict(type(train_cfg)())
    tc["runner"]["num_steps_per_env"] = steps_per_env
    runner = OnPolicyRunner(env, tc, None, device="cpu")
    runner.learn(1)  # warm
    t0 = time.time()
    runner.learn(1)
    dt = time.time() - t0
    return steps_per_env * n_envs / dt, dt


# SURVEY.md 8(d) CPU-baseline plan: C1 (64 envs) and C2 (4096 envs flat) besides the bench's C3
# workload, at the CPU share of the box and at 1 thread.  A sample is one PPO iteration; the
# throughput of an iteration does not depend on its length (collection and learn both scale with
# the sample count), so the 1-thread runs of the large configs use fewer steps per env to keep the
# whole baseline at ~1 minute of CPU time.
CPU_RUNS = [  # (label, task, envs, steps per env at full share, steps per env at 1 thread)
    ("C1", "go1_flat_bench", 64, 24, 24),
    ("C2", "go1_flat_bench", 4096, 24, 2),
    ("C3", "go1_rough", 4096, 24, 1),
]


def cpu_baseline(task, n_envs):
    """The C oracle env + torch-CPU PPO ("port": the reference CPU path needs Isaac Gym, absent),
    timed on this host at the configs of CPU_RUNS; value = the bench workload's config (C3) at the
    full CPU share.  threads = the CPUs this job may use: OMP_NUM_THREADS (the GPU box's per-GPU
    CPU share), else the affinity set, capped by the physical cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    info = _host_cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or info["affinity_cpus"]
    if info.get("physical_cores"):
        share = min(share, info["physical_cores"])
    runs = []
    t_all = time.time()
    for label, t, n, spe_full, spe_one in CPU_RUNS:
        if label == "C3":
            t, n = task, n_envs
        for threads, spe in ((share, spe_full), (1, spe_one)):
            v, dt = _cpu_iteration(t, n, spe, threads)
            runs.append({"config": label, "task": t, "envs": n, "steps_per_env": spe, "threads": threads,
                         "value": v, "seconds": round(dt, 3)})
    head = next(r for r in runs if r["config"] == "C3" and r["threads"] == share)
    return dict(value=head["value"], unit="env-steps/s", cores=share, kind="port",
                sample=f"1 PPO iteration ({head['steps_per_env']} steps x {head['envs']} envs, {head['task']}) of the C "
                       f"oracle env (OpenMP over envs: physics, actuator net, rewards, observations) + torch-CPU "
                       f"ActorCritic/PPO, {share} threads; `runs` adds C1 / C2 and 1-thread runs "
                       f"({time.time() - t_all:.0f} s of baseline in total, warm-ups included)",
                runs=runs, host=info)


# LGX_BENCH_POSTHOC=0: skip the launches bench.py times after the timed region (the isolated dW and
# standalone actuator-net launches), so that a rocprofv3 --stats summary of the run holds in-situ
# launches only (tools/gpu_profile.sh prof step)
POSTHOC = os.environ.get("LGX_BENCH_POSTHOC", "1") != "0"


def isolated_tn(fused, torch, reps=20):
    """(algorithmic FLOP, ms, launches) of the update's dW launches (lgx_gemm_tn with the last
    minibatch's arguments) run alone on the current stream after the timed region."""
    import ctypes as C
    dw = getattr(fused, "gemm_dw", None)
    if not dw:
        return None
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    flop = ms = 0.0
    n = 0
    for k in sorted(dw):
        for t in dw[k]:
            for _ in range(3):
                fused.check(fused.lib.lgx_gemm_tn(C.byref(t), stream), "gemm_tn")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fused.check(fused.lib.lgx_gemm_tn(C.byref(t), stream), "gemm_tn")
            e1.record()
            e1.synchronize()
            ms += e0.elapsed_time(e1)
            n += reps
            flop += reps * 2.0 * t.M * t.R * t.Cc * t.batch
    return flop, ms, n


def standalone_actuator_ms(lib, env, torch, launches=50):
    """Average duration of the standalone actuator-net launch over the env's current model_ins."""
    stream = torch.cuda.current_stream()
    x, y = env._model_ins_all, torch.empty_like(env._actuator_dvel)
    rows = x.numel() // 30

    def launch():
        lib.lgx_actuator_mlp(C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), rows,
                             C.c_void_p(env.actuator_net_weights.data_ptr()),
                             C.c_void_p(env.actuator_net_scale.data_ptr()), C.c_void_p(stream.cuda_stream))
    for _ in range(5):
        launch()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(launches):
        launch()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / launches, launches


def param_fingerprint(flat, torch):
    """Exact integer fingerprint of a float32 parameter vector: sum of its bit patterns x (index
    mod 1021 + 1), in int64 (no overflow below 4e6 parameters) - equal on two ranks iff their
    parameters are bitwise equal (up to a collision of this weighted sum)."""
    bits = flat.detach().contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 1021 + 1
    return (bits * w).sum()


def data_parallel_check(runner, fused, comm_t, world, backend, device, dist):
    """After the timed region: what a multi-GPU run has to prove from its own JSON line - the ranks
    that took part, that every rank ends with bitwise identical parameters (fingerprint MAX - MIN
    over ranks == 0), whether the two-bucket gradient all-reduce ran (FusedPPOUpdate.bucketed), and
    the event-timed all-reduce time per iteration (the timed minibatches, scaled)."""
    import torch
    alg = runner.alg
    flat = fused.flat_p if fused is not None else torch.cat([p.detach().reshape(-1) for p in alg.actor_critic.parameters()])
    fp = param_fingerprint(flat, torch).view(1)
    out = {"world": world, "backend": backend, "param_fingerprint": int(fp.item())}
    if dist is not None:
        hi, lo, ranks = fp.clone(), fp.clone(), torch.ones(1, dtype=torch.int64, device=device)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(ranks)
        out.update(ranks_seen=int(ranks.item()), param_fingerprint_spread=int((hi - lo).item()),
                   params_identical_across_ranks=bool((hi == lo).item()))
    if fused is not None:
        out["bucketed_allreduce"] = bool(fused.bucketed)
        out["join_events"] = fused.join_events   # cross-stream joins: "system" whenever data-parallel
        out["allreduce_impl"] = fused.allreduce_impl   # "lgx" = lgx_allreduce_grads (LGX_NATIVE_ALLREDUCE=1)
        n, ms, nbytes, mbs = comm_t
        mb_per_iter = alg.num_learning_epochs * alg.num_mini_batches
        out["allreduce"] = {"collectives_timed": n, "bytes_per_minibatch": (nbytes / mbs) if mbs else 0,
                            "ms_per_iteration": (ms / mbs * mb_per_iter) if mbs else 0.0,
                            "note": "HIP events around every gradient all-reduce of every k-th minibatch "
                                    "(LGX_BENCH_GEMM_TIMING), on the stream it is issued from"}
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus n > 1 without a launcher: run this script as n ranks under torch.distributed.run in a
    child process (never exec: nothing here has touched the GPU, and the child owns the ranks),
    stdout passed through (rank 0 prints the JSON line); returns the launcher's exit code, non-zero
    when any rank failed."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


def rendezvous_check(world, rank):
    """--rendezvous_only: the ranks' gloo rendezvous on CPU (no GPU touched); returns the rank's
    exit code."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    seen = torch.ones(1)
    if world > 1:
        dist.all_reduce(seen)
        dist.barrier()
    if rank == 0:
        print(json.dumps({"rendezvous": "gloo", "world": world, "ranks_seen": int(seen.item())}))
        sys.stdout.flush()
    fail = os.environ.get("LGX_BENCH_FAIL_RANK")
    code = 3 if fail is not None and int(fail) == rank else 0
    if world > 1:
        dist.destroy_process_group()
    return code


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least one GPU")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}: "
                         "one rank per GPU, the two must agree")
    if args.actuator_net_torques and not args.task.startswith("anymal"):
        raise SystemExit("--actuator_net_torques: the SEA actuator network is ANYmal's (anymal.py:71-78); "
                         f"task {args.task} has no actuator-net torque source")
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rendezvous_only:
        sys.exit(rendezvous_check(world, rank))
    # one rank per GPU (identity on a full node); LGX_DIST_BACKEND=gloo with more ranks than GPUs
    # rehearses the data-parallel path on a single device
    backend = os.environ.get("LGX_DIST_BACKEND", "nccl")
    ngpu = torch.cuda.device_count() if backend != "nccl" else 0
    if ngpu:
        local = local % ngpu
    # LGX_DIST_REHEARSAL=1 (under torch.distributed.run, one rank): the data-parallel path - process
    # group, parameter broadcast, bucketed gradient all-reduce, the self-check - over a one-rank
    # communicator, on the one GPU of a test box
    distributed = world > 1 or os.environ.get("LGX_DIST_REHEARSAL") == "1"
    if distributed:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    device = f"cuda:{local}"
    import legged_gym_amd.envs  # noqa: F401
    from legged_gym_amd.sim import lib as lgxlib
    from legged_gym_amd.utils.helpers import get_args
    from legged_gym_amd.utils.task_registry import task_registry

    env_cfg, train_cfg = task_registry.get_cfgs(args.task)
    env_cfg = type(env_cfg)()
    train_cfg = type(train_cfg)()
    env_cfg.env.num_envs = args.num_envs
    if args.actuator_net_torques:
        env_cfg.control.explicit_torques = True
    env_cfg.seed = 1 + rank
    train_cfg.seed = 1 + rank
    cli = get_args(["--sim_device", device, "--rl_device", device, "--headless", "--task", args.task])
    env, _ = task_registry.make_env(args.task, args=cli, env_cfg=env_cfg)
    runner, _ = task_registry.make_alg_runner(env, name=args.task, args=cli, train_cfg=train_cfg, log_root=None)
    from legged_gym_amd.sim import abi
    ctrl = {v: k for k, v in abi.CTRL.items()}.get(env._control_type(), "?")
    if args.actuator_net_torques and ctrl != "SEA":
        raise SystemExit(f"--actuator_net_torques: {args.task} resolved control type {ctrl}, not the SEA network "
                         "(needs cfg.control.use_actuator_network)")
    lib = lgxlib.load()
    handle = env._backend.handle

    runner.learn(args.warmup)
    gc.collect()
    gc.disable()   # no collector pauses inside the timed region (host-side Python only)
    timing_period = int(os.environ.get("LGX_BENCH_KERNEL_TIMING", "7"))   # time every k-th env step (0: off); 7 is coprime with the 24-step rollout, so every step position (the cold first one included) is sampled in proportion
    lib.lgx_profile_enable(handle, timing_period)
    fused = getattr(runner.alg, "_fused", None)
    if fused is not None:   # HIP events around the PPO-update GEMM launches of every k-th minibatch
        fused.time_gemms(int(os.environ.get("LGX_BENCH_GEMM_TIMING", "7")))
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.learn(args.steps)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    lib.lgx_profile_enable(handle, 0)
    gemm_t = fused.gemm_timings() if fused is not None else {}
    comm_t = fused.comm_timings() if fused is not None else None
    if fused is not None:
        fused.time_gemms(0)
    ms = (C.c_double * 3)()
    cnt = (C.c_int64 * 3)()
    lgxlib.check(lib.lgx_profile_collect(handle, ms, cnt), "lgx_profile_collect")
    if distributed:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    data_parallel = data_parallel_check(runner, fused, comm_t, world, backend if distributed else None, device,
                                        dist if distributed else None)
    N = args.num_envs
    steps_per_iter = runner.num_steps_per_env
    value = steps_per_iter * N * world * args.steps / elapsed

    # roofline of the dominant lgx kernel (HIP-event durations over the timed region)
    fused_act = hasattr(env, "_actuator_dvel") and cnt[1] == 0
    names = ["lgx_physics_kernel", "lgx_actuator_ws_kernel",
             "lgx_post_physics_act_kernel" if fused_act else "lgx_post_physics_kernel"]
    avg = [ms[i] / cnt[i] if cnt[i] else 0.0 for i in range(3)]
    act_note = None
    if fused_act:
        # the actuator net shares the post-physics launch in the rollout; its own roofline is
        # measured on the same rows with the standalone launch (after the timed region)
        avg[1], launches = standalone_actuator_ms(lib, env, torch) if POSTHOC else (0.0, 0)
        act_note = (f"standalone lgx_actuator_ws_kernel on this step's model_ins rows, {launches} launches after the "
                    "timed region (in the rollout it runs on workgroups of lgx_post_physics_act_kernel)")
    decim = env.cfg.control.decimation
    phys_flop = N * decim * physics_flop_per_env_substep(
        env._lgx_model.num_points, 4.0, env.cfg.terrain.mesh_type in ("heightfield", "trimesh"))
    roof = {"kernel": names[0], "bound": "valu", "compute_pipe": "fp32 VALU",
            "achieved": (phys_flop / (avg[0] * 1e-3) / 1e12) if avg[0] else None,
            "peak": MI355X_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "traffic": pmc_traffic_bytes(f"lgx_physics_kernel<{lib.lgx_physics_lane_split(N)}>", args.task, N),
            "algorithmic_per_launch": phys_flop,
            "note": ("compute roof = FP32 peak (vector FP32 = f32 MFMA = 157.3 TF on gfx950); algorithmic FLOP "
                     "from legged_gym_amd/sim/flops.py x envs x substeps; traffic = FETCH_SIZE*2 + WRITE_SIZE "
                     "per launch from " + os.path.relpath(PMC_FILE, ROOT) + " (tools/gpu_profile.sh; null when that file was "
                     "collected on another workload); latency-bound, see DESIGN.md 4.1")}
    act_flop = ACT_MLP_FLOP_PER_ENV_STEP * N
    roof2 = {"kernel": "lgx_actuator_ws_kernel", "bound": "mfma", "peak": MI355X_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
             "achieved": (act_flop / (avg[1] * 1e-3) / 1e12) if avg[1] else None,
             "traffic": pmc_traffic_bytes("lgx_actuator_ws_kernel", args.task, N, "fetch_sep", "write_sep"),
             "algorithmic_per_launch": act_flop}
    if act_note:
        roof2["note"] = act_note
    for r in (roof, roof2):
        if r["achieved"] is not None:
            r["frac"] = r["achieved"] / r["peak"]
    it_ms = 1000.0 * elapsed / args.steps
    # the PPO-update GEMM instantiations, timed live (events on the launch stream)
    mb_per_iter = runner.alg.num_learning_epochs * runner.alg.num_mini_batches
    gemm_roofs = []
    for epi, (n, t_ms, flop, mbs) in sorted(gemm_t.items(), key=lambda kv: str(kv[0])):
        if not n or not mbs:
            continue
        kname, pipe, peak = gemm_kernel_info(epi, getattr(fused, "split", False))
        gemm_roofs.append({
            "kernel": kname, "bound": "mfma", "compute_pipe": pipe,
            "achieved": flop / (t_ms * 1e-3) / 1e12, "peak": peak, "unit": "TFLOP/s",
            "frac": flop / (t_ms * 1e-3) / 1e12 / peak,
            "traffic": pmc_ppo_traffic_bytes(kname, args.task, N), "algorithmic_per_launch": flop / n,
            "avg_ms": t_ms / n, "mfma": pmc_mfma_busy(kname, args.task, N),
            "launches_timed": n, "share_of_iteration": (t_ms / mbs) * mb_per_iter / it_ms,
            "note": GEMM_NOTES.get(epi, "") + "; algorithmic FLOP = 2 M N K x {actor, critic} with the unpadded K / Cc "
                    "(f32 products; the split-bf16 peak is the bf16 dense MFMA peak / 6 limb products); HIP events "
                    "around every launch of every k-th minibatch (LGX_BENCH_GEMM_TIMING); traffic = 2 FETCH_SIZE + "
                    f"WRITE_SIZE per launch from {os.path.relpath(PPO_PMC_FILE, ROOT)}"})
        if epi == "tn" and getattr(fused, "_side", None) is not None:
            # dW runs on the update's second stream next to dA: its launches overlap
            # dA's, so their durations are co-resident times and their share is not exclusive
            gemm_roofs[-1]["concurrent"] = True
            gemm_roofs[-1]["note"] += ("; launched on a second stream concurrently with the dA GEMMs: durations "
                                       "are co-resident times (the CUs are shared), not the isolated kernel rate")
            iso = isolated_tn(fused, torch) if POSTHOC else None
            if iso:
                f_iso, ms_iso, n_iso = iso
                gemm_roofs[-1]["isolated"] = {
                    "achieved": f_iso / (ms_iso * 1e-3) / 1e12, "frac": f_iso / (ms_iso * 1e-3) / 1e12 / peak,
                    "avg_ms": ms_iso / n_iso, "launches": n_iso,
                    "note": "the same dW launches (last minibatch's arguments) alone on the main stream after the "
                            "timed region, HIP events; the kernel's own rate without the co-resident dA GEMMs"}
    kernels = {n: {"avg_ms": round(a, 4), "launches_timed": int(c),
                   "share_of_iteration": round(a * steps_per_iter / it_ms, 4) if c else None}
               for n, a, c in zip(names, avg, cnt)}
    # `roofline` = the lgx kernel with the largest GPU-time share of the iteration, kernels that run
    # concurrently on the update's second stream included (their share is co-resident GPU time);
    # the others follow in `roofline_others`, in the same order
    phys_share = avg[0] * steps_per_iter / it_ms      # one launch per env step (timing is sampled)
    roof["share_of_iteration"] = phys_share
    cands = [roof] + gemm_roofs
    cands.sort(key=lambda r: -r.get("share_of_iteration", 0.0))
    roof, others = cands[0], cands[1:]
    if roof.get("mfma"):
        roof["mfma_busy"] = roof["mfma"]["mfma_busy"]
    roof["selection"] = ("largest GPU-time share of the iteration among the physics kernel and the PPO-update GEMM "
                         "families (second-stream launches included)")
    out = {
        "metric": (BASELINE_METRIC if (args.task == "go1_rough" and N == 4096)
                   else f"env-steps/sec (whole node), {args.task} {N} envs/GPU"),
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": it_ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32", "data": "synthetic (procedural curriculum terrain, random-init policy)",
        "config": {"workload": WORKLOADS.get(args.task, args.task) +
                               (", SEA actuator-net torques" if ctrl == "SEA" else "") +
                               f", PPO {steps_per_iter} steps x {N} envs/GPU, "
                               f"{runner.alg.num_learning_epochs} epochs x {runner.alg.num_mini_batches} minibatches",
                   "envs_per_gpu": N, "global_envs": N * world, "parallelism": f"dp{world}"},
        "roofline": roof,
        "roofline_others": others,
        "roofline_secondary": roof2,
        "iteration_roofline": iteration_roofline(runner, env, N, it_ms),
        "dominant_lgx_kernel": roof["kernel"],
        "lgx_kernels": kernels,
        "mfma_utilisation": {k: pmc_mfma_busy(k, args.task, N) for k in MFMA_KERNELS},
        "last_iteration": runner.last_iteration_stats,
        "data_parallel": data_parallel,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.task, args.cpu_envs)
        except Exception as e:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out))
    if distributed:
        runner.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
