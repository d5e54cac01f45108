#!/bin/bash
# A/B variant of liblgx: build/ab/<name>/liblgx.so from the same sources with extra compiler
# flags (e.g. -DX3_INTERLEAVE=0).  CPU side; select with LGX_LIB_PATH=build/ab/<name>/liblgx.so.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/ab/$name
for f in legged_gym_amd/csrc/*.hip; do
  case $(basename $f) in   # the product build's per-file flags (legged_gym_amd/csrc/Makefile)
    lgx_physics.hip|lgx_gemm_split.hip|lgx_gemm_x3p.hip|lgx_gemm_tn.hip|lgx_mlp_x3.hip) ff=-fno-slp-vectorize ;;
    *) ff= ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics $ff "$@" \
    -c $f -o build/ab/$name/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab/$name/liblgx.so build/ab/$name/*.o
