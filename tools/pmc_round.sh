#!/bin/bash
# PMC counter passes (rocprofv3 --pmc with --kernel-trace only; one counter group per pass).
# Target: the env-step kernels under tools/kbench.py physrun (go1_rough, 4096 envs, 10 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "list failed"; exit 1; }
want="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM"
have=""
for c in $want; do grep -qw "$c" $OUT/avail.txt && have="$have $c"; done
echo "valu counters:$have"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python tools/kbench.py physrun > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -20 $OUT/$name.log; return 1; }
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run valu $have && LGX_PHYS_PP=1 run valu_pp1 $have
rc=$?
find $OUT -name "*counter_collection*" | head
exit $rc
