#!/bin/bash
# PPO-update kernel stats (rocprofv3 --kernel-trace --stats over tools/host_overhead.py), for the
# tree's liblgx.so and (A/B) build/ab/head/liblgx.so on the same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ddp.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || { echo "ppo tests rc=$?"; tail -30 gpurun_out/ppo_tests.log; exit 1; }
tail -1 gpurun_out/ppo_tests.log
for v in head new head new; do
  if [ $v = head ]; then export LGX_LIB_PATH=build/ab/head/liblgx.so; else unset LGX_LIB_PATH; fi
  rm -rf gpurun_out/prof_$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run --output-format csv -- python3 tools/host_overhead.py > gpurun_out/prof_$v.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/prof_$v.log; exit 1; }
  echo "$v: $(grep -h 'adam_clip\|sumsq' gpurun_out/prof_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | tr '\n' ' ')"
done
