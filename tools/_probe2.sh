#!/bin/bash
# rollout MLP A/B: x3 parity tests, timing + phase clocks, then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo.py -x -q -m gpu -k "x3 or rollout or mlp" --timeout 120 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { echo "x3 tests rc=$?"; tail -30 gpurun_out/x3_tests.log; exit 1; }
tail -2 gpurun_out/x3_tests.log
timeout -k 10 120 python -u tools/ubench_x3.py > gpurun_out/ubench_x3.log 2>&1 || { echo "ubench_x3 rc=$?"; tail -20 gpurun_out/ubench_x3.log; exit 1; }
grep "x3 actor" gpurun_out/ubench_x3.log
LGX_LIB_PATH=build/clock/liblgx.so timeout -k 10 120 python -u tools/ubench_x3.py > gpurun_out/ubench_x3_clock.log 2>&1 || { echo "clock rc=$?"; tail -20 gpurun_out/ubench_x3_clock.log; exit 1; }
grep -m 3 "cycles" gpurun_out/ubench_x3_clock.log
timeout -k 10 600 python bench.py --no_cpu_baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bench.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['last_iteration'])
"
