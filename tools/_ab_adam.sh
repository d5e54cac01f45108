#!/bin/bash
# same-box A/B of the PPO update: build/ab/head (previous Adam kernels) vs the tree's liblgx.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ddp.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || { echo "ppo tests rc=$?"; tail -30 gpurun_out/ppo_tests.log; exit 1; }
tail -1 gpurun_out/ppo_tests.log
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export LGX_LIB_PATH=build/ab/head/liblgx.so; else unset LGX_LIB_PATH; fi
    timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/ab_$v.log 2>&1 || { echo "$v rc=$?"; tail -20 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep 'update rep\|rep 2:' gpurun_out/ab_$v.log | tr '\n' ' ')"
  done
done
