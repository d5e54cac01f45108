"""bench.py's launch contract on CPU: --gpus N > 1 without a launcher starts N
ranks itself under torch.distributed.run (a child process) and exits with the launcher's code; a
launcher-provided WORLD_SIZE that disagrees with --gpus is refused before any work.  On this
GPU-less host every rank fails at its first device call, which is exactly what shows that both
ranks were started and that the failure reaches the exit code (the successful two-rank run is
tests/test_gpu_ddp.py::test_bench_plain_gpus2_launches_ranks)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], cwd=ROOT,
                       env=_env(WORLD_SIZE="3"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr and "--gpus 2" in r.stderr


def test_gpus_zero_is_refused():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-only check (ranks fail without a GPU)")
def test_plain_gpus2_starts_two_ranks_and_propagates_failure():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no_cpu_baseline"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "torch.distributed" in r.stderr
    assert "local_rank: 0" in r.stderr and "local_rank: 1" in r.stderr


def _rendezvous(fail_rank=None):
    env = _env(OMP_NUM_THREADS="1")
    if fail_rank is not None:
        env["LGX_BENCH_FAIL_RANK"] = str(fail_rank)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rendezvous_only"], cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=300)


def test_launch_ranks_gloo_two_ranks_succeed():
    """Plain `bench.py --gpus 2` (no launcher): launch_ranks starts two ranks, they rendezvous over
    gloo on CPU, both are counted, and the launcher exits 0."""
    import json
    r = _rendezvous()
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert json.loads(line[-1]) == {"rendezvous": "gloo", "world": 2, "ranks_seen": 2}


@pytest.mark.parametrize("fail_rank", [1, 0])
def test_launch_ranks_returns_a_failing_ranks_code(fail_rank):
    """One of two gloo ranks exits non-zero after a successful rendezvous (the other exits 0):
    launch_ranks, hence `bench.py --gpus 2`, exits non-zero."""
    r = _rendezvous(fail_rank)
    assert r.returncode != 0, r.stdout + r.stderr[-2000:]
    assert '"ranks_seen": 2' in r.stdout     # the failure came after both ranks had joined
