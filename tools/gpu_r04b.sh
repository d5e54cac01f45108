#!/bin/bash
# Round-4 GPU session B: Cassie / dense physics kernel tests, derived-tolerance physics tests,
# golden replays (incl. cassie_rough), then a Cassie bench and a rocprof of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "cassie or dense or physics_substeps or rough_terrain_derived" \
  > gpurun_out/r04b_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04b_tests.log | tail -30
if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "tests aborted rc=$rc"; exit 1; fi
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_golden.py > gpurun_out/r04b_golden.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04b_golden.log | tail -15
if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "golden aborted rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --task cassie --steps 5 --warmup 2 --no_cpu_baseline > gpurun_out/r04b_cassie_bench.json 2> gpurun_out/r04b_cassie_bench.err || { echo "cassie bench failed"; tail -20 gpurun_out/r04b_cassie_bench.err; exit 1; }
tail -1 gpurun_out/r04b_cassie_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cassie', round(d['value']/1e6,4), 'M env-steps/s', round(d['ms_per_step'],2), 'ms/it', d['lgx_kernels'])"
timeout -k 10 200 python tools/phys_bench.py go1_rough 4096 50 > gpurun_out/r04b_phys.log 2>&1 || { echo "phys bench failed"; tail -5 gpurun_out/r04b_phys.log; exit 1; }
cat gpurun_out/r04b_phys.log | grep physics
LGX_LIB_PATH=build/clock/liblgx.so timeout -k 10 200 python tools/phys_bench.py go1_rough 4096 3 > gpurun_out/r04b_phys_clock.log 2>&1 || { echo "clock bench failed"; tail -5 gpurun_out/r04b_phys_clock.log; exit 1; }
grep "physics cycles" gpurun_out/r04b_phys_clock.log | tail -3
