#!/bin/bash
# same-box A/B of the rollout MLP: build/ab/head (previous kernel) vs the tree's liblgx.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo.py -x -q -m gpu -k "x3 or rollout or mlp" --timeout 120 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { echo "x3 tests rc=$?"; tail -30 gpurun_out/x3_tests.log; exit 1; }
tail -1 gpurun_out/x3_tests.log
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export LGX_LIB_PATH=build/ab/head/liblgx.so; else unset LGX_LIB_PATH; fi
    timeout -k 10 120 python -u tools/ubench_x3.py > gpurun_out/ab_$v.log 2>&1 || { echo "$v rc=$?"; tail -20 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep 'x3 actor' gpurun_out/ab_$v.log | tr '\n' ' ')"
  done
done
