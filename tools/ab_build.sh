#!/bin/bash
# A/B variant of liblgx: tools/_tmp/ab/<name>/liblgx.so from the same sources with extra compiler
# flags (e.g. -DX3P_BOLD=0).  CPU side; select with LGX_LIB_PATH=tools/_tmp/ab/<name>/liblgx.so
# (git-ignored, not gpurun-ignored: it travels to the GPU box).  AB_ONLY=<source basename> rebuilds
# only that object and links it with the product objects (seconds instead of a full build).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=tools/_tmp/ab/$name
mkdir -p $out
C=legged_gym_amd/csrc
flags_for() {   # the product build's per-file flags (legged_gym_amd/csrc/Makefile)
  case $(basename $1) in
    lgx_physics.hip|lgx_gemm_split.hip|lgx_gemm_x3p.hip|lgx_gemm_tn.hip|lgx_mlp_x3.hip) echo -fno-slp-vectorize ;;
  esac
}
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics"
if [ -n "$AB_ONLY" ]; then
  make -C $C -s -j8 >/dev/null
  $HIPCC $(flags_for $AB_ONLY.hip) "$@" -c $C/$AB_ONLY.hip -o $out/$AB_ONLY.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/liblgx.so $(ls $C/*.o | grep -v "/$AB_ONLY.o") $out/$AB_ONLY.o
  exit 0
fi
for f in $C/*.hip; do
  $HIPCC $(flags_for $f) "$@" -c $f -o $out/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/liblgx.so $out/*.o
