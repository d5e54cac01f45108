set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "4 0" "16 0" "8 1" "8 0"; do set -- $cfg
LGX_MLP_WAVES=$1 LGX_CRITIC_OVERLAP=$2 timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/bench_w$1_o$2.json 2>/dev/null
done
