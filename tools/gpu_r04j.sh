#!/bin/bash
# Side-stream priority A/B (LGX_PPO_SIDE_PRIO: 0 = normal, -1 = high) on the bench, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for r in 1 2 3; do
  for v in 0 -1; do
    LGX_PPO_SIDE_PRIO=$v timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no_cpu_baseline > gpurun_out/r04j_$v.json 2> gpurun_out/r04j.err || { echo "$v failed"; tail -5 gpurun_out/r04j.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); li=d['last_iteration']; print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms learn', round(li['learn_time']*1e3,2), 'coll', round(li['collection_time']*1e3,2))" gpurun_out/r04j_$v.json $v
  done
done
