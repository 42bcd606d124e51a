#!/bin/bash
# GPU-box runner: each step under its own timeout; stop at the first step that
# crashes, faults or times out (rc other than 0/1).  Logs under gpurun_out/.
mkdir -p gpurun_out
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n "${TAILN:-4}" "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run gpu_tests 900 python -m pytest tests -m gpu -q -x ;;
    tests_all) run gpu_tests 900 python -m pytest tests -m gpu -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_gather) run bench_gather 600 python bench.py --ft-impl gather --no-cpu-baseline ;;
    bench_games) run bench_games 600 python bench.py --workload games --no-cpu-baseline ;;
    bench_children) run bench_children 600 python bench.py --workload children --games 1000 --no-cpu-baseline ;;
    profile) run profile 1200 tools/profile.sh "${PROFILE_TAG:-rXX}" ;;
    profile_gather) run profile_gather 1200 tools/profile.sh "${PROFILE_TAG:-rXX}_gather" --ft-impl gather ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
