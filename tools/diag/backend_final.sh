#!/bin/bash
# GPU box: the engine actor's closing evidence — its bench line (1 / 64 / 1024 /
# 16384 batches per go(), CPU baseline), the HIP/kernel trace of 40 steady calls
# at 1 and 1024 batches with their timelines and trace summary, and the host
# marks (FNNUE_BACKEND_TRACE) of one run.
#   usage: tools/diag/backend_final.sh <tag>
set -uo pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 400 python bench.py --workload backend > "$out/bench_backend.log" 2>&1 || { tail -5 "$out/bench_backend.log"; exit 1; }
grep '^{' "$out/bench_backend.log" | tail -1 > "$out/bench_backend.json"
bash tools/backend_trace.sh "$tag" 1,1024 40 || exit 1
T=gpurun_out/btrace_$tag/trace
python tools/diag/backend_timeline.py $T 0 > "$out/timeline_1batch.txt" || exit 1
python tools/diag/backend_timeline.py $T 1 > "$out/timeline_1024batches.txt" || exit 1
python tools/diag/backend_trace_summary.py $T 40 1 1024 > "$out/trace_summary.txt" || exit 1
FNNUE_BACKEND_TRACE=1 timeout -k 10 200 python bench.py --workload backend --go-batches 1,1024,16384 --go-calls 40 \
  --no-cpu-baseline > "$out/marks_bench.json" 2> "$out/marks.txt" || exit 1
