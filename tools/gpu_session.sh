#!/bin/bash
# Bench instrumentation overhead: kernel / GEMM event sampling periods (same box, alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for r in 1 2; do
  for v in "7 7" "0 0" "13 13"; do
    set -- $v
    LGX_BENCH_KERNEL_TIMING=$1 LGX_BENCH_GEMM_TIMING=$2 timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bt.json 2> gpurun_out/bt.err || { echo "bench failed"; tail -5 gpurun_out/bt.err; exit 1; }
    echo "periods $1/$2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bt.json)"
  done
done
