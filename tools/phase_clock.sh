#!/bin/bash
# Build an instrumented copy of liblgx (per-phase clock64 sums of block 0 / thread 0, printed by
# the kernels) into tools/_tmp/clock/ — run on the CPU side; use with LGX_LIB_PATH=tools/_tmp/clock/liblgx.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_tmp/clock
for f in legged_gym_amd/csrc/*.hip; do
  case $(basename $f) in   # the product build's per-file flags (legged_gym_amd/csrc/Makefile)
    lgx_physics.hip|lgx_gemm_split.hip|lgx_gemm_x3p.hip|lgx_gemm_tn.hip|lgx_mlp_x3.hip) ff=-fno-slp-vectorize ;;
    *) ff= ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $ff -DLGX_PHASE_CLOCK ${CLK_EXTRA:-} -c $f -o tools/_tmp/clock/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/_tmp/clock/liblgx.so tools/_tmp/clock/*.o
