#!/bin/bash
# Same-box A/B of whole-iteration throughput: HEAD vs an older tree copied under build/old_tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
ROOT=$PWD
for r in 1 2 3; do
  for v in head old; do
    if [ $v = old ]; then cd $ROOT/build/old_tree; else cd $ROOT; fi
    timeout -k 10 300 python bench.py --no_cpu_baseline > $ROOT/gpurun_out/ab_$v.json 2> $ROOT/gpurun_out/ab_$v.err || { echo "$v failed"; tail -5 $ROOT/gpurun_out/ab_$v.err; exit 1; }
    echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $ROOT/gpurun_out/ab_$v.json) $(grep -o '"collection_time": [0-9.]*' $ROOT/gpurun_out/ab_$v.json) $(grep -o '"learn_time": [0-9.]*' $ROOT/gpurun_out/ab_$v.json)"
  done
done
