#!/bin/bash
# PMC counter passes (rocprofv3 --pmc with --kernel-trace only; one counter group per pass).
# Target: the env-step kernels under tools/kbench.py physrun (go1_rough, 4096 envs, 10 steps);
# the *_sep passes run the actuator net as its own launch (LGX_ACT_OVERLAP=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf $OUT; mkdir -p $OUT
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python tools/kbench.py physrun > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -20 $OUT/$name.log; return 1; }
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
  LGX_ACT_OVERLAP=0 LGX_ACT_X3=0 run fetch_sep FETCH_SIZE && LGX_ACT_OVERLAP=0 LGX_ACT_X3=0 run write_sep WRITE_SIZE && \
  run valu SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32
rc=$?
python tools/pmc_summary.py $OUT gpurun_out/pmc_env_kernels.json > /dev/null || rc=1
exit $rc
