set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_def.json 2>/dev/null
LGX_ACT_WS_PER_CU=1 timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_def1.json 2>/dev/null
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_L.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs -o run --output-format csv -- python tools/kbench.py physrun > gpurun_out/pcs.log 2>&1
