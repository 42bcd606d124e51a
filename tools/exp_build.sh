#!/bin/bash
# Builds an experimental variant of libfnnue.so with extra -D flags on the HIP
# sources (ft_sliced.hip and kernels.hip) into exp/libfnnue_<name>.so (run
# bench with FNNUE_LIB=...).
#   usage: tools/exp_build.sh <name> [-DFLAG ...]
set -euo pipefail
cd "$(dirname "$0")/../fishnet_amd/csrc"
make -s -j8
name=$1; shift
mkdir -p ../../exp build/exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c ft_sliced.hip -o build/exp/ft_sliced_$name.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c kernels.hip -o build/exp/kernels_$name.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/libfnnue_$name.so \
  build/board.o build/net.o build/capi.o build/exp/kernels_$name.o build/exp/ft_sliced_$name.o -lpthread
echo "exp/libfnnue_$name.so"
