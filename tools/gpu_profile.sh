#!/bin/bash
# One GPU session of profiles for a round (replaces the per-session gpu_r04*.sh / pmc_*.sh scripts):
#   tools/gpu_profile.sh <round tag, e.g. r05> [steps...]
# steps (default: all, in this order):
#   envpmc  - env-step kernels under tools/kbench.py physrun (go1_rough, 4096 envs): stall and
#             instruction counters, HBM FETCH/WRITE, the actuator net on its own launch (*_sep)
#   ppopmc  - one bench iteration's PPO-update and rollout kernels: HBM FETCH/WRITE and MFMA
#             utilisation (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...)
#   bench   - bench.py with the fresh PMC files (-> gpurun_out/<tag>_bench.json)
#   prof    - rocprofv3 --kernel-trace --stats of bench.py --steps 5 (-> gpurun_out/<tag>_prof), without
#             bench.py's post-timed isolated dW / standalone actuator launches (LGX_BENCH_POSTHOC=0):
#             every kernel average in the summary is an in-situ figure
# One --pmc counter group per pass, --kernel-trace only; every GPU step has its own time limit and
# the first failure ends the session.  BENCH_ARGS / LGX_PMC_TASK / LGX_PMC_ENVS select another
# workload (e.g. BENCH_ARGS="--task anymal_c_rough --num_envs 8192" LGX_PMC_TASK=anymal_c_rough
# LGX_PMC_ENVS=8192).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
TAG=${1:?round tag}; shift
STEPS=${*:-envpmc ppopmc bench prof}
export LGX_PMC_TASK=${LGX_PMC_TASK:-go1_rough} LGX_PMC_ENVS=${LGX_PMC_ENVS:-4096}
BENCH_ARGS=${BENCH_ARGS:-}
mkdir -p gpurun_out
run() {  # out dir, name, target (phys|bench), counters...
  local dir=$1 name=$2 tgt=$3; shift 3
  if [ $tgt = phys ]; then
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $dir/$name -o run --output-format csv -- python tools/kbench.py physrun > $dir/$name.log 2>&1
  else
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" -d $dir/$name -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no_cpu_baseline $BENCH_ARGS > $dir/$name.log 2>&1
  fi
  local rc=$?
  [ $rc = 0 ] || { echo "pass $name failed rc=$rc"; tail -20 $dir/$name.log; return 1; }
}
for step in $STEPS; do
  case $step in
  envpmc)
    O=gpurun_out/${TAG}_pmc_env; rm -rf $O; mkdir -p $O
    run $O stall phys SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT && \
    run $O inst phys SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 && \
    run $O fetch phys FETCH_SIZE && run $O write phys WRITE_SIZE && \
    LGX_ACT_OVERLAP=0 run $O fetch_sep phys FETCH_SIZE && \
    LGX_ACT_OVERLAP=0 run $O write_sep phys WRITE_SIZE || exit 1
    python tools/pmc_summary.py $O gpurun_out/${TAG}_pmc_env_kernels.json "rocprofv3 --kernel-trace --pmc, per-dispatch means over tools/kbench.py physrun (go1_rough, 4096 envs, 10 env steps); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide coalesced bytes); SQ_* cycle counters per dispatch summed over SEs (DESIGN 4.1); passes *_sep ran with LGX_ACT_OVERLAP=0 (actuator net as its own launch), instruction counters = wave-instructions per dispatch" > /dev/null || exit 1 ;;
  ppopmc)
    O=gpurun_out/${TAG}_pmc_ppo; rm -rf $O; mkdir -p $O
    run $O fetch bench FETCH_SIZE && run $O write bench WRITE_SIZE && \
    run $O mfma bench SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit 1
    python tools/pmc_summary.py $O gpurun_out/${TAG}_pmc_ppo_kernels.json "rocprofv3 --kernel-trace --pmc, per-dispatch means over bench.py --steps 1 --warmup 1 (${LGX_PMC_TASK}, ${LGX_PMC_ENVS} envs: 2 PPO iterations; rocprofv3 serialises dispatches under --pmc, so the second-stream kernels run alone); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide coalesced bytes); pass mfma: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs), GRBM_GUI_ACTIVE (cycles summed over the 8 XCDs), SQ_* instruction counts per dispatch" > /dev/null || exit 1 ;;
  bench)
    export LGX_BENCH_PMC_ENV=$PWD/gpurun_out/${TAG}_pmc_env_kernels.json LGX_BENCH_PMC_PPO=$PWD/gpurun_out/${TAG}_pmc_ppo_kernels.json
    [ -f $LGX_BENCH_PMC_ENV ] || unset LGX_BENCH_PMC_ENV
    [ -f $LGX_BENCH_PMC_PPO ] || unset LGX_BENCH_PMC_PPO
    timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
    cat gpurun_out/${TAG}_bench.json ;;
  prof)
    rm -rf gpurun_out/${TAG}_prof
    LGX_BENCH_POSTHOC=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no_cpu_baseline $BENCH_ARGS > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo "prof failed"; tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
    find gpurun_out/${TAG}_prof -name "*stats*" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
