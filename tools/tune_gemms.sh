#!/bin/bash
# Re-tune the PPO-update GEMMs on the GPU box with torch TunableOp and refresh the shipped table.
#   gpurun -- 'bash tools/tune_gemms.sh'  then copy gpurun_out/tune/ppo_gemms_gfx950.csv to
#   legged_gym_amd/resources/tunableop/
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/tune
export LGX_TUNED_GEMMS=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/ppo_gemms_gfx950.csv
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --no_cpu_baseline > gpurun_out/tune/tune_bench.json 2> gpurun_out/tune/tune.err
