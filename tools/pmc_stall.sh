#!/bin/bash
# Where the env-step kernels' wave time goes: SQ cycle counters (one pass, --kernel-trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc_stall
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "list failed"; exit 1; }
want="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
have=""
for c in $want; do grep -qw "$c" $OUT/avail.txt && have="$have $c"; done
echo "counters:$have"
set -- $have
g1="$1 $2 $3 $4 $5 $6 $7 $8"; shift 8 2>/dev/null
g2="$*"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $g1 -d $OUT/p1 -o run --output-format csv -- python tools/kbench.py physrun > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail -20 $OUT/p1.log; exit 1; }
if [ -n "$g2" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $g2 -d $OUT/p2 -o run --output-format csv -- python tools/kbench.py physrun > $OUT/p2.log 2>&1 || { echo "p2 failed"; tail -20 $OUT/p2.log; exit 1; }
fi
find $OUT -name "*counter_collection*"
