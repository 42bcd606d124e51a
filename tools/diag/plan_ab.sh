#!/bin/bash
# GPU box: A/B of plan-kernel variants (tools/exp_build.sh libraries) on the
# grouped workloads and the engine actor's small / medium calls.
#   usage: tools/diag/plan_ab.sh <tag> <variant ...>
set -uo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
WLS=${WLS:-"games children crazyhouse-games"} ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash tools/exp_run.sh "$@" > "$out/ab.txt" 2>&1 || exit 1
cat "$out/ab.txt"
for r in 1 2; do
  for v in main "$@"; do
    lib=$PWD/exp/libfnnue_$v.so; [ $v = main ] && lib=$PWD/fishnet_amd/libfnnue.so
    FNNUE_LIB=$lib timeout -k 10 200 python bench.py --workload backend --go-batches ${GO:-1,64,1024} --go-calls 200 \
      --no-cpu-baseline > "$out/backend_${v}_$r.json" 2>/dev/null || exit 1
    python tools/diag/abtab_one.py $v "$out/backend_${v}_$r.json"
  done
done
