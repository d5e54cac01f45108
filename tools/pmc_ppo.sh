#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per rocprofv3 --pmc pass,
# --kernel-trace only) over one bench.py iteration: the PPO-update kernels (lgx_gemm_nt, loss,
# reductions) in situ -> profiles/r03_pmc_ppo_kernels.json (read by bench.py's roofline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ppo
rm -rf $OUT; mkdir -p $OUT
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no_cpu_baseline > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -20 $OUT/$name.log; return 1; }
}
run fetch FETCH_SIZE && run write WRITE_SIZE || exit 1
python tools/pmc_summary.py $OUT gpurun_out/pmc_ppo_kernels.json "rocprofv3 --kernel-trace --pmc, per-dispatch means over bench.py --steps 1 --warmup 1 (go1_rough, 4096 envs: 2 PPO iterations); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide coalesced bytes)" > /dev/null
