#!/bin/bash
# Physics A/B: HEAD build vs the working tree on go1_rough 4096 and anymal_c_rough 8192; phase clocks;
# the physics parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for task in "go1_rough 4096" "anymal_c_rough 8192"; do
  for r in 1 2; do
    for v in head default; do
      if [ $v = default ]; then unset LGX_LIB_PATH; else export LGX_LIB_PATH=$PWD/build/ab/$v/liblgx.so; fi
      timeout -k 10 200 python tools/phys_bench.py $task 50 > gpurun_out/r04h_phys_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r04h_phys_$v.log; exit 1; }
      echo "$v: $(grep physics gpurun_out/r04h_phys_$v.log)"
    done
  done
done
unset LGX_LIB_PATH
LGX_LIB_PATH=build/clock/liblgx.so timeout -k 10 200 python tools/phys_bench.py go1_rough 4096 3 > gpurun_out/r04h_phys_clock.log 2>&1 || { echo "clock bench failed"; tail -5 gpurun_out/r04h_phys_clock.log; exit 1; }
grep "physics cycles" gpurun_out/r04h_phys_clock.log | tail -2
env ${TEST_LIB:+LGX_LIB_PATH=$TEST_LIB} timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_terrain.py tests/test_gpu_golden.py \
  > gpurun_out/r04h_tests.log 2>&1
grep -E "FAIL|Error|passed|failed" gpurun_out/r04h_tests.log | tail -30
