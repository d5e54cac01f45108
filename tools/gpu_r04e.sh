#!/bin/bash
# Round-4 profiles: physics stall attribution (SQ wait / LDS / VALU counters), env-kernel HBM
# traffic, PPO-kernel traffic, the bench line and the rocprofv3 kernel-trace summary of the same
# build.  One --pmc counter group per pass, --kernel-trace only; every GPU step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/pmc04
rm -rf $OUT; mkdir -p $OUT
run() {  # name, target, counters...
  local name=$1 tgt=$2; shift 2
  if [ $tgt = phys ]; then
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python tools/kbench.py physrun > $OUT/$name.log 2>&1
  else
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no_cpu_baseline > $OUT/$name.log 2>&1
  fi
  local rc=$?
  [ $rc = 0 ] || { echo "pass $name failed rc=$rc"; tail -20 $OUT/$name.log; return 1; }
}
run stall phys SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT && \
run inst phys SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 && \
run fetch phys FETCH_SIZE && run write phys WRITE_SIZE && \
  LGX_ACT_OVERLAP=0 LGX_ACT_X3=0 run fetch_sep phys FETCH_SIZE && LGX_ACT_OVERLAP=0 LGX_ACT_X3=0 run write_sep phys WRITE_SIZE || exit 1
python tools/pmc_summary.py $OUT gpurun_out/r04_pmc_env_kernels.json "rocprofv3 --kernel-trace --pmc, per-dispatch means over tools/kbench.py physrun (go1_rough, 4096 envs, 10 env steps); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide coalesced bytes); SQ_* cycle counters per dispatch summed over SEs (see DESIGN 4.1); passes *_sep ran with LGX_ACT_OVERLAP=0 (actuator net as its own launch), instruction counters = wave-instructions per dispatch" > /dev/null || exit 1
OUT=gpurun_out/pmc04_ppo
rm -rf $OUT; mkdir -p $OUT
run fetch bench FETCH_SIZE && run write bench WRITE_SIZE || exit 1
python tools/pmc_summary.py $OUT gpurun_out/r04_pmc_ppo_kernels.json "rocprofv3 --kernel-trace --pmc, per-dispatch means over bench.py --steps 1 --warmup 1 (go1_rough, 4096 envs: 2 PPO iterations); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide coalesced bytes)" > /dev/null || exit 1
export LGX_BENCH_PMC_ENV=$PWD/gpurun_out/r04_pmc_env_kernels.json LGX_BENCH_PMC_PPO=$PWD/gpurun_out/r04_pmc_ppo_kernels.json
timeout -k 10 600 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { echo "bench failed"; tail -20 gpurun_out/r04_bench.err; exit 1; }
cat gpurun_out/r04_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof04 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no_cpu_baseline > gpurun_out/r04_prof_bench.json 2> gpurun_out/r04_prof.err || { echo "prof failed"; tail -20 gpurun_out/r04_prof.err; exit 1; }
find gpurun_out/prof04 -name "*stats*"
