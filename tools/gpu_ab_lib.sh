#!/bin/bash
# Kernel-time A/B of library variants (tools/_tmp/ab/<name>/liblgx.so via LGX_LIB_PATH) on the env
# kernels: rocprofv3 stats of tools/kbench.py physrun (go1_rough, 4096 envs), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in default $AB_VARIANTS; do
    if [ $v = default ]; then unset LGX_LIB_PATH; else export LGX_LIB_PATH=$PWD/tools/_tmp/ab/$v/liblgx.so; fi
    rm -rf gpurun_out/ab_$v
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- python tools/kbench.py physrun > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep -h -E 'lgx_physics_kernel<4>|lgx_post_physics_act_kernel' gpurun_out/ab_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1,3 | tr '\n' ' ')"
  done
done
