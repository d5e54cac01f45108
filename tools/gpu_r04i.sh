#!/bin/bash
# dW row-slice sweep (LGX_PPO_SPLITS per hidden layer), alternated bench runs on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for r in 1 2; do
  for v in default 16,32,32 16,16,16 8,16,32 16,8,32 32,32,32; do
    if [ $v = default ]; then unset LGX_PPO_SPLITS; else export LGX_PPO_SPLITS=$v; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no_cpu_baseline > gpurun_out/r04i_$v.json 2> gpurun_out/r04i.err || { echo "$v failed"; tail -5 gpurun_out/r04i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); li=d['last_iteration']; print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms learn', round(li['learn_time']*1e3,2), 'coll', round(li['collection_time']*1e3,2))" gpurun_out/r04i_$v.json $v
  done
done
