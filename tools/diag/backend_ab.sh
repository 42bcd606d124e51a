#!/bin/bash
# A/B of the backend actor's host/device schedule knobs (GPU box, repo root):
#   tools/diag/backend_ab.sh <tag> "<ENV=.. ENV=..>" ...   one bench run per argument
# each: --workload backend at 1 / 1024 / 16384 batches per go(), with the
# host timeline (FNNUE_BACKEND_TRACE) in trace_<i>.txt
set -uo pipefail
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for cfg in "$@"; do
  echo "$cfg" > "$out/cfg_$i.txt"
  env $cfg FNNUE_BACKEND_TRACE=1 timeout -k 10 200 python bench.py --workload backend --go-batches 1,1024,16384 \
    --go-calls 40 --no-cpu-baseline > "$out/bench_$i.json" 2> "$out/trace_$i.txt" || exit 1
  i=$((i + 1))
done
