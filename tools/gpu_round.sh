#!/bin/bash
# GPU-box round check: the -m gpu suite, smoke(), then one bench line per
# workload; every GPU step under its own timeout, stop at the first failure.
# Logs / JSON under gpurun_out/$ROUND_TAG.
set -o pipefail
O=gpurun_out/${ROUND_TAG:-rXX}; mkdir -p $O
STEPS=${STEPS:-"tests smoke positions games children crazyhouse atomic"}
for st in $STEPS; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
        || { echo "tests rc=$?"; tail -40 $O/gputest.log; exit 1; }
      tail -2 $O/gputest.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    positions|games|children|crazyhouse|atomic|crazyhouse-games|atomic-games|devices)
      a="--workload $st"; [ $st = devices ] && a="--launch devices --gpus 1"
      timeout -k 10 400 python bench.py $a $BENCH_ARGS > $O/bench_$st.json 2> $O/bench_$st.err \
        || { echo "bench $st rc=$?"; tail -20 $O/bench_$st.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench_$st.json'));r=d['roofline'];print('$st', d['config']['positions_per_gpu'], round(d['value']/1e6,1), round(d['ms_per_step'],3), r['frac'], r['bound'], r['plan_avg_ms'], r['kernel_avg_ms'], r['stack_kernel_avg_ms'], round((d['cpu_baseline'] or {}).get('value',0)/1e6,2), d['parity_spot_check'], (d['gathered'] or {}).get('gather_ms'))" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
