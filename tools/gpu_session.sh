#!/bin/bash
# Ad-hoc GPU session: runner / PPO / parity tests, then the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_ppo.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ppo_tests.log; exit 1; }
tail -1 gpurun_out/ppo_tests.log
timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || { echo "bench failed"; tail -20 gpurun_out/bench_s.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"collection_time": [0-9.]*' gpurun_out/bench_s.json | head -3
LGX_DEFER_STORE=0 timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_s0.json 2> gpurun_out/bench_s0.err || { echo "bench failed"; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"collection_time": [0-9.]*' gpurun_out/bench_s0.json | head -3
