#!/bin/bash
# GPU box: kernel-trace stats of bench.py for experimental libraries
#   usage: tools/prof_exp.sh name1 name2 ...  -> per-kernel average ns
export TMPDIR=/tmp
for v in "$@"; do
  out=$PWD/gpurun_out/pexp/$v
  mkdir -p "$out"
  FNNUE_LIB=$PWD/exp/libfnnue_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$out/log" 2>&1 || exit 3
  python3 - "$out/run_kernel_stats.csv" "$v" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
parts = []
for r in rows:
    m = re.search(r"(\w+_kernel)", r["Name"])
    if m and not m.group(1).startswith("vectorized") and m.group(1) != "relayout_kernel":
        parts.append(f"{m.group(1).replace('_kernel','')}={float(r['AverageNs'])/1e3:.1f}us")
print(f"{sys.argv[2]:14s} " + " ".join(parts))
PY
done
