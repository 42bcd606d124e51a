#!/bin/bash
# GPU box: the engine actor's bench (small and medium calls) per library
# variant (tools/exp_build.sh), alternating, ROUNDS times.
#   usage: GO=1,8,64,1024 tools/diag/backend_lib_ab.sh <tag> <variant ...>   (main = in-tree library)
set -uo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    lib=$PWD/exp/libfnnue_$v.so; [ $v = main ] && lib=$PWD/fishnet_amd/libfnnue.so
    FNNUE_LIB=$lib timeout -k 10 200 python bench.py --workload backend --go-batches ${GO:-1,8,64,1024} --go-calls 200 \
      --no-cpu-baseline > "$out/backend_${v}_$r.json" 2>/dev/null || exit 1
    python tools/diag/abtab_one.py $v "$out/backend_${v}_$r.json"
  done
done
