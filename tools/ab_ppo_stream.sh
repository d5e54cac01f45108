#!/bin/bash
# Same-box A/B of the PPO update's backward stream schedule (one full update at the bench shape per
# run): default (two cross-stream syncs per minibatch) vs LGX_PPO_SCHED=0 (four).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "LGX_PPO_SCHED=2" "LGX_PPO_SCHED=0"; do
    echo "== [$v]"
    env $v timeout -k 10 120 python tools/kbench.py ppo_lgx 2>&1 | grep "PPO update" || exit 1
  done
done
