#!/bin/bash
# Builds an experimental variant of libfnnue.so with extra -D flags on every
# HIP source (the tunables FT_UNIT_ITEMS, SEG_UNIT_PLIES, PLAN_WG, FT_DEPTH;
# knock-out experiments are patched into a scratch copy, never the shipped
# sources)
# into exp/libfnnue_<name>.so (run bench with FNNUE_LIB=...).
#   usage: tools/exp_build.sh <name> [-DFLAG ...]
set -euo pipefail
cd "$(dirname "$0")/../fishnet_amd/csrc"
make -s -j8
name=$1; shift
mkdir -p ../../exp build/exp
objs=""
for src in *.hip; do
  o=build/exp/${src%.hip}_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c $src -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/libfnnue_$name.so \
  build/board.o build/net.o build/capi.o build/multi.o build/variant_host.o build/backend.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -lpthread
echo "exp/libfnnue_$name.so"
