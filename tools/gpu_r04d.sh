#!/bin/bash
# Round-4 GPU session D: exact-f32 MFMA dW (LGX_GEMM_TN_F32=1) vs the split-bf16 dW kernel:
# GEMM tests, isolated kernel rates at the update shapes, the whole bench alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "gemm_tn" \
  > gpurun_out/r04d_gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r04d_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r04d_gemm_tests.log
KB_SLICES=8,16,32 timeout -k 10 200 python tools/kbench.py tn > gpurun_out/r04d_tn_split.log 2>&1 || { tail -5 gpurun_out/r04d_tn_split.log; exit 1; }
LGX_GEMM_TN_F32=1 KB_SLICES=8,16,32 timeout -k 10 200 python tools/kbench.py tn > gpurun_out/r04d_tn_f32.log 2>&1 || { tail -5 gpurun_out/r04d_tn_f32.log; exit 1; }
echo split; grep gemm_tn gpurun_out/r04d_tn_split.log
echo f32; grep gemm_tn gpurun_out/r04d_tn_f32.log
for r in 1 2; do
  for v in split f32; do
    if [ $v = f32 ]; then export LGX_GEMM_TN_F32=1; else unset LGX_GEMM_TN_F32; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no_cpu_baseline > gpurun_out/r04d_bench_${v}_$r.json 2> gpurun_out/r04d_bench.err || { tail -5 gpurun_out/r04d_bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['frac'],3), 'learn', d.get('last_iteration',{}).get('learn_time'))" gpurun_out/r04d_bench_${v}_$r.json $v
  done
done
