#!/bin/bash
# Kernel-time A/B of library variants (tools/_tmp/ab/<name>/liblgx.so via LGX_LIB_PATH) on the PPO
# update's GEMMs: rocprofv3 stats of tools/kbench.py ppo_lgx (one full update), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in default $AB_VARIANTS; do
    if [ $v = default ]; then unset LGX_LIB_PATH; else export LGX_LIB_PATH=$PWD/tools/_tmp/ab/$v/liblgx.so; fi
    rm -rf gpurun_out/abp_$v
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$v -o run --output-format csv -- python tools/kbench.py ppo_lgx > gpurun_out/abp_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abp_$v.log; exit 1; }
    echo "$v: $(grep 'PPO update' gpurun_out/abp_$v.log) | $(grep -h -E 'gemm_nt_x3p|gemm_tn_' gpurun_out/abp_$v/run_kernel_stats.csv | awk -F'",' '{print $1 "|" $2}' | sed 's/.*kernel<//; s/>((anonymous namespace)::[A-Za-z]*Args)//' | cut -d, -f1,3 | tr '\n' ' ')"
  done
done
