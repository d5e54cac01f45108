#!/bin/bash
# Ad-hoc GPU session: PPO tests, then an in-process A/B of LGX_PPO_SQ.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ddp.py tests/test_gpu_runner.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || { echo "ppo tests failed"; tail -40 gpurun_out/ppo_tests.log; exit 1; }
tail -3 gpurun_out/ppo_tests.log
KB_VAR=LGX_PPO_SQ KB_VALUES=1,0 bash tools/ab_ppo_stream.sh
