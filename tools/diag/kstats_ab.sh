#!/bin/bash
# GPU box: rocprofv3 kernel stats of one bench workload per library variant.
#   usage: tools/diag/kstats_ab.sh <tag> <workload> <variant ...>   (main = the in-tree library)
set -uo pipefail
tag=$1; wl=$2; shift 2
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/exp/libfnnue_$v.so; [ $v = main ] && lib=$PWD/fishnet_amd/libfnnue.so
  FNNUE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v" -o run -- \
    python3 bench.py --workload $wl --steps 30 --no-cpu-baseline --no-host-api > "$out/$v.log" 2>&1 || exit 1
  python3 - "$out/$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("fnnue::", "").split("(")[0]
    print(f"{sys.argv[2]:8s} {n[:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
