#!/bin/bash
# SQ counters of the hand-written PPO-update GEMMs (lgx_gemm_nt), one --pmc pass per group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
g1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
g2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g1 -d $OUT/p1 -o run --output-format csv -- python3 tools/kbench.py gemm > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g2 -d $OUT/p2 -o run --output-format csv -- python3 tools/kbench.py gemm > $OUT/p2.log 2>&1 || { echo "p2 failed"; tail -20 $OUT/p2.log; exit 1; }
find $OUT -name "*counter_collection*"
