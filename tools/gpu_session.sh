#!/bin/bash
# Loss+backward rows per workgroup A/B: kernel averages under rocprofv3 (one PPO update), the
# default library vs build/ab/lb16 (-DLGX_LB_ROWS=16); then the lb16 library's PPO tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default lb16 default lb16; do
  if [ $v = lb16 ]; then export LGX_LIB_PATH=$PWD/build/ab/lb16/liblgx.so; else unset LGX_LIB_PATH; fi
  rm -rf gpurun_out/p_$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p_$v -o run --output-format csv -- python tools/kbench.py ppo_lgx > gpurun_out/p_$v.log 2>&1 || { echo "prof $v failed"; tail -5 gpurun_out/p_$v.log; exit 1; }
  echo "$v: $(grep 'PPO update' gpurun_out/p_$v.log)"
  grep -h -E "ppo_loss_bwd|reduce_slices" gpurun_out/p_$v/run_kernel_stats.csv | cut -d, -f1-4
done
LGX_LIB_PATH=$PWD/build/ab/lb16/liblgx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lb16_tests.log 2>&1; echo "lb16 tests rc=$?"; tail -1 gpurun_out/lb16_tests.log
