#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of one bench.py run (args passed through);
# prints per-kernel average microseconds.  FNNUE_LIB may select a variant.
#   usage: tools/prof_kernels.sh <tag> [bench args...]
export TMPDIR=/tmp
tag=$1; shift
out=$PWD/gpurun_out/pk/$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-api "$@" > "$out/log" 2>&1 || exit 3
python3 - "$out/run_kernel_stats.csv" "$tag" <<'PY'
import csv, re, sys
parts = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(\w+_kernel)", r["Name"])
    name = m.group(1) if m else r["Name"][:30]
    parts.append(f"{name.replace('_kernel','')}={float(r['AverageNs'])/1e3:.1f}us x{r['Calls']}")
print(f"{sys.argv[2]:14s} " + " ".join(parts))
PY
