#!/bin/bash
# Round-4 GPU session A: the new / changed GPU tests, the physics error probe (HIP and float32
# oracle vs the float64 oracle), then a short bench A/B of the dW row slices (default 16/16/32 vs
# dW1 sized for all CUs: 32/16/32), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/physics_err_probe.py > gpurun_out/r04a_probe.jsonl 2> gpurun_out/r04a_probe.err || { echo "probe failed rc=$?"; tail -20 gpurun_out/r04a_probe.err; }
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ppo.py::test_fused_update_bench_shape_every_step_is_exact \
  tests/test_gpu_fullsize.py::test_full_size_subset_matches_oracle \
  tests/test_gpu_parity.py::test_physics_substeps_match_oracle tests/test_gpu_parity.py::test_physics_rough_terrain_derived_tolerance \
  tests/test_gpu_parity.py::test_anymal_sea_torque_step_matches_oracle \
  tests/test_gpu_parity.py::test_gae_kernel_matches_torch_loop tests/test_gpu_parity.py::test_gae_norm_large_mean_advantages \
  tests/test_gpu_golden.py tests/test_gpu_ddp.py > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04a_tests.log | grep -E "PASS|FAIL|Error|passed|failed" | tail -25
if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "tests aborted rc=$rc"; exit 1; fi
for i in 1 2; do
  for S in default 32,16,32; do
    if [[ $S == default ]]; then unset LGX_PPO_SPLITS; else export LGX_PPO_SPLITS=$S; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/r04a_bench_${S}_$i.json 2> gpurun_out/r04a_bench.err || { echo "bench failed"; tail -20 gpurun_out/r04a_bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,4), round(d['ms_per_step'],3), d['last_iteration']['collection_time'], d['last_iteration']['learn_time'])" gpurun_out/r04a_bench_${S}_$i.json $S
  done
done
