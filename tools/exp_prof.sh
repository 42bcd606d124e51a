#!/bin/bash
# GPU box: kernel-trace stats of bench runs per experimental variant
# (tools/exp_build.sh): per-kernel average durations side by side.
#   usage: tools/exp_prof.sh name1 name2 ...   (extra bench args in $BENCH_ARGS)
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for v in "$@"; do
  FNNUE_LIB=$PWD/exp/libfnnue_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/exp/prof_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/exp/prof_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/exp/prof_$v.log; exit $rc; }
  f=$(find gpurun_out/exp/prof_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    import re; m = re.search(r"(\w+_kernel|\w+Kernel\w*|__amd\w+)", r["Name"]); name = (m.group(1) if m else r["Name"])[:40]
    if int(r["Calls"]) >= 10:
        print(f"  {name:40s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
done
