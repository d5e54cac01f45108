"""GPU micro-benchmark of the physics launch at a bench size (default C3: go1_rough, 4096 envs):
the env is stepped with random actions for a realistic state (robots standing / walking / fallen on
the curriculum terrain), then `decimation` substeps of the physics kernel are timed with HIP events
on the launch stream.  With LGX_LIB_PATH pointing at a phase-clock build (tools/phase_clock.sh) the
kernel prints per-phase cycle sums of block 0 / thread 0 for the last launches.

Usage: python tools/phys_bench.py [task] [num_envs] [launches]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from oracle_backend import make_env  # noqa: E402


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "go1_rough"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    launches = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    env = make_env(task, num_envs=n, device="cuda:0", backend="lgx")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(30):
        env.step(torch.randn(n, 12, device="cuda:0", generator=g) * 0.5)
    torch.cuda.synchronize()
    dec = env.cfg.control.decimation
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(launches):
        env.simulate(dec)
    e.record()
    e.synchronize()
    print(f"{task} {n} envs: physics launch ({dec} substeps) {1000 * s.elapsed_time(e) / launches:.1f} us", flush=True)


if __name__ == "__main__":
    main()
