#!/bin/bash
# One GPU-box session: tests, bench, rocprof kernel trace.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEP == all || $STEP == prof ]]; then
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no_cpu_baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
