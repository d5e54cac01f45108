#!/bin/bash
# probes after the round tests/bench: update host issue time, rollout MLP timing + phase clocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/host_overhead.log 2>&1 || { echo "host_overhead rc=$?"; tail -20 gpurun_out/host_overhead.log; exit 1; }
cat gpurun_out/host_overhead.log | grep -v Warn
timeout -k 10 120 python -u tools/ubench_x3.py > gpurun_out/ubench_x3.log 2>&1 || { echo "ubench_x3 rc=$?"; tail -20 gpurun_out/ubench_x3.log; exit 1; }
cat gpurun_out/ubench_x3.log
LGX_LIB_PATH=build/clock/liblgx.so timeout -k 10 120 python -u tools/ubench_x3.py > gpurun_out/ubench_x3_clock.log 2>&1 || { echo "clock rc=$?"; tail -20 gpurun_out/ubench_x3_clock.log; exit 1; }
grep -m 12 "cycles\|x3 actor" gpurun_out/ubench_x3_clock.log
