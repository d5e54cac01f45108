"""One-rank RCCL rehearsal of bench.py per LGX_NATIVE_ALLREDUCE value given on the command line
(e.g. `python tools/allreduce_ab.py 0 1 0 1`): prints the all-reduce implementation, the parameter
fingerprint, the event-timed all-reduce ms per iteration and ms per iteration.
AB_TASK / AB_ENVS / AB_STEPS select the workload (default go1_flat_bench, 1024 envs, 2 steps)."""
import json, os, socket, subprocess, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p
for native in sys.argv[1:]:
    env = dict(os.environ, LGX_DIST_BACKEND="nccl", LGX_DIST_REHEARSAL="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               LGX_BENCH_GEMM_TIMING="1", LGX_NATIVE_ALLREDUCE=native)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", os.environ.get("AB_STEPS", "2"), "--warmup", "1",
           "--task", os.environ.get("AB_TASK", "go1_flat_bench"), "--num_envs", os.environ.get("AB_ENVS", "1024"),
           "--no_cpu_baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    dp = d["data_parallel"]
    print(native, dp["allreduce_impl"], dp["param_fingerprint"], dp["allreduce"]["ms_per_iteration"], d["ms_per_step"], flush=True)
