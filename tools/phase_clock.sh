#!/bin/bash
# Build an instrumented copy of liblgx (per-phase clock64 sums of block 0 / thread 0, printed by
# the kernels) into build/clock/ — run on the CPU side; use with LGX_LIB_PATH=build/clock/liblgx.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/clock
for f in legged_gym_amd/csrc/*.hip; do
  case $(basename $f) in   # the product build's per-file flags (legged_gym_amd/csrc/Makefile)
    lgx_physics.hip|lgx_gemm_split.hip|lgx_gemm_x3p.hip|lgx_gemm_tn.hip|lgx_mlp_x3.hip) ff=-fno-slp-vectorize ;;
    *) ff= ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $ff -DLGX_PHASE_CLOCK ${CLK_EXTRA:-} -c $f -o build/clock/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/clock/liblgx.so build/clock/*.o
