#!/bin/bash
# GPU box: the round's closing evidence on the final tree, in one call, each
# step under its own time limit, stopping at the first step that fails:
#   1. the whole GPU suite and smoke()
#   2. rocprofv3 kernel trace + PMC passes of every bench workload, including
#      the small net's width (games@128, positions@128): profile_round.sh
#   3. those counters installed into THIS box's profiles/counters.json
#      (roofline.py --install; the tree hash is the sources', identical here),
#      so that
#   4. the bench lines of every workload carry counters.tree_matches = true.
# Everything lands in gpurun_out/<tag>/ (copy counters.json back into
# profiles/ on the build machine).
#   usage: tools/final_round.sh <tag> [phase ...]   phases: tests profile bench (default: all)
# (one gpurun call may last 20 minutes: run the phases in two calls if needed;
# the bench phase installs the profile phase's counters first)
set -uo pipefail
tag=${1:-rXX}
shift || true
phases=${*:-tests profile bench}
has() { [[ " $phases " == *" $1 "* ]]; }
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -n 2 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
if has tests; then
  step gputest 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has profile; then
  step profile 1800 bash tools/profile_round.sh "$tag" positions games children crazyhouse atomic crazyhouse-games \
    atomic-games games@128 positions@128
fi
has bench || exit 0
# counters of this call's profile phase; in a call of its own the bench phase
# uses the profiles/counters.json installed from them on the build machine
# (gpurun_out/ does not travel to the next box)
[ -d "gpurun_out/prof_$tag" ] && step install 120 python tools/roofline.py "gpurun_out/prof_$tag" --install
cp profiles/counters.json "$out/counters.json"
b() {  # b <name> <bench args...>
  local name=$1; shift
  step "bench_$name" 400 python bench.py --steps 200 "$@"
  grep '^{' "$out/bench_$name.log" | tail -1 > "$out/bench_$name.json"
}
b positions
b games --workload games --no-host-api
b games_small --workload games --small-net 128 --no-host-api
b children --workload children --no-host-api
b crazyhouse --workload crazyhouse --no-host-api
b atomic --workload atomic --no-host-api
b crazyhouse-games --workload crazyhouse-games --no-host-api
b atomic-games --workload atomic-games --no-host-api
b games_small_nodual --workload games --small-net 128 --no-dual --no-host-api
b backend --workload backend
