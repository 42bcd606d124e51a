#!/bin/bash
# rocprofv3 evidence for a bench workload (run on the GPU box from the repo root):
#   kernel trace + stats, then one PMC pass per counter group (never combined
#   with tracing domains).  Outputs under gpurun_out/prof_<tag>/.
#   usage: tools/profile.sh <tag> [extra bench.py args...]
#   env: PMCS="set1|set2|..." (space-separated counters per set), SKIP_TRACE=1
set -uo pipefail
TAG=${1:-rXX}; shift || true
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${SKIP_TRACE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-api "$@" > "$OUT/trace.log" 2>&1
  rc=$?
  echo "trace rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
PMCS=${PMCS:-"FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
IFS='|' read -ra SETS <<< "$PMCS"
for pmc in "${SETS[@]}"; do
  name=$(echo "$pmc" | tr ' ' '_' | cut -c1-60)
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc_$name" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-api "$@" > "$OUT/pmc_$name.log" 2>&1
  rc=$?
  echo "pmc [$pmc] rc=$rc"
  # a counter the hardware rejects fails fast (rc 1); anything else ends the run
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt"
echo "profile done: $OUT"
