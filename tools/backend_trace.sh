#!/bin/bash
# rocprofv3 evidence for the backend actor (run on the GPU box from the repo
# root): HIP API + kernel trace with stats over exactly N steady-state
# fnnue_backend_go calls per batch count (after warm-up calls), so the trace
# shows what one go() enqueues, allocates and waits for.
#   usage: tools/backend_trace.sh <tag> <batches-per-go,...> [calls]
set -uo pipefail
TAG=${1:-rXX}
SIZES=${2:-1,1024}
CALLS=${3:-100}
OUT=$PWD/gpurun_out/btrace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d "$OUT/trace" -o run -- python3 bench.py --workload backend --go-batches "$SIZES" --go-calls "$CALLS" \
  --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/trace.log"
rc=$?
echo "trace rc=$rc"
exit $rc
