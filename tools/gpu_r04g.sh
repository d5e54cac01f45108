#!/bin/bash
# Physics lane split at C5 (anymal_c_rough, 8192 envs: two rounds of waves at PP = 4, one at PP = 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for r in 1 2; do
  for pp in 4 2; do
    LGX_PHYS_PP=$pp timeout -k 10 200 python tools/phys_bench.py anymal_c_rough 8192 50 > gpurun_out/r04g_pp$pp.log 2>&1 || { echo "pp$pp failed"; tail -5 gpurun_out/r04g_pp$pp.log; exit 1; }
    echo "pp$pp: $(grep physics gpurun_out/r04g_pp$pp.log)"
  done
done
