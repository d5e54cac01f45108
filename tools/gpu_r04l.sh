#!/bin/bash
# HIP_FORCE_DEV_KERNARG A/B (kernel arguments in device memory) on the bench, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for r in 1 2; do
  for v in unset 1 0; do
    if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no_cpu_baseline > gpurun_out/r04l_$v.json 2> gpurun_out/r04l.err || { echo "$v failed"; tail -5 gpurun_out/r04l.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); li=d['last_iteration']; print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms learn', round(li['learn_time']*1e3,2), 'coll', round(li['collection_time']*1e3,2))" gpurun_out/r04l_$v.json $v
  done
done
