#!/bin/bash
# Ad-hoc GPU session: runner tests, bench, stream-schedule A/B, RCCL probe (each step time-limited).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py -x -v --timeout 120 --timeout-method thread > gpurun_out/runner_tests.log 2>&1 || { echo "runner tests failed"; tail -30 gpurun_out/runner_tests.log; exit 1; }
tail -3 gpurun_out/runner_tests.log
timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_defer.json 2> gpurun_out/bench_defer.err || { echo "bench failed"; tail -20 gpurun_out/bench_defer.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_defer.json')); print('bench', d['value'], d['ms_per_step'], d['last_iteration'] if 'last_iteration' in d else '')"
bash tools/ab_ppo_stream.sh || exit 1
timeout -k 10 90 python tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "rccl probe rc=$?"; tail -5 gpurun_out/rccl_probe.log
