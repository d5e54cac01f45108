#!/bin/bash
# Ad-hoc GPU session: PPO tests (both backward schedules), then the schedule A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ddp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || { echo "ppo tests failed"; tail -40 gpurun_out/ppo_tests.log; exit 1; }
tail -3 gpurun_out/ppo_tests.log
bash tools/ab_ppo_stream.sh
