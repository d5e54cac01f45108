set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LGX_BENCH_KERNEL_TIMING=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no_cpu_baseline > gpurun_out/prof1.json 2> gpurun_out/prof1.err
for k in 0 1 8; do LGX_BENCH_KERNEL_TIMING=$k timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_t$k.json 2>/dev/null; done
