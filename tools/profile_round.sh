#!/bin/bash
# GPU box: rocprofv3 evidence of the current tree for the bench workloads
# (config 2 positions, config 3 games, config 4 children at its per-GPU scale,
# config 5 crazyhouse / atomic), each with bench.py's default sizes:
#   trace/   kernel trace + stats (one run)
#   pmc_<k>/ one PMC pass per counter set, each its own run (never combined
#            with tracing domains; every set within the per-block limits)
# then tools/roofline.py turns them into gpurun_out/prof_<tag>/counters.json.
#   usage: tools/profile_round.sh <tag> [workload ...]   (default: all of them)
# A workload "<name>@<hd>" profiles bench.py --workload <name> --hd <hd>
# (counters keyed so; bench.py reads them for that width, e.g. the small net);
# "backend:<k>" profiles the engine actor at <k> batches per go().
set -uo pipefail
TAG=${1:-rXX}; shift || true
WLS=${*:-positions games children crazyhouse atomic crazyhouse-games atomic-games}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
)
for wl in $WLS; do
  args="--workload ${wl%@*}"
  [[ $wl == *@* ]] && args="$args --hd ${wl#*@}"
  # backend:<k>: the engine actor at <k> acquired batches per go() (bench.py --workload backend)
  [[ $wl == backend:* ]] && args="--workload backend --go-batches ${wl#backend:} --go-calls 20"
  D=$OUT/$wl
  mkdir -p "$D"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --settle-s 0 --no-cpu-baseline --no-host-api --no-extra $args > "$D/trace.log" 2>&1
  rc=$?
  echo "[$wl trace] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=0
  for pmc in "${SETS[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$D/pmc_$i" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --settle-s 0 --no-cpu-baseline --no-host-api --no-extra $args > "$D/pmc_$i.log" 2>&1
    rc=$?
    echo "[$wl pmc $i: $pmc] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/roofline.py "$OUT" > "$OUT/roofline.txt" && cat "$OUT/roofline.txt"
