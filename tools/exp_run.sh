#!/bin/bash
# GPU box: bench each experimental variant (tools/exp_build.sh) once.
#   usage: tools/exp_run.sh name1 name2 ...   (extra bench args in $BENCH_ARGS)
mkdir -p gpurun_out/exp
for v in "$@"; do
  FNNUE_LIB=$PWD/exp/libfnnue_$v.so timeout -k 10 300 python bench.py --cpu-seconds 1 --no-host-api ${BENCH_ARGS:-} \
    > gpurun_out/exp/$v.log 2>&1
  rc=$?
  python3 - "$v" "$rc" <<'PY'
import json, sys
v, rc = sys.argv[1], sys.argv[2]
try:
    line = [l for l in open(f"gpurun_out/exp/{v}.log") if l.startswith("{")][-1]
    d = json.loads(line)
    print(f"{v:12s} rc={rc} {d['value']/1e6:8.1f}M/s plan={d['roofline']['plan_avg_ms']:.4f} ft={d['roofline']['kernel_avg_ms']:.4f} ms stack={d['roofline']['stack_kernel_avg_ms']:.4f} mism={(d.get('parity_spot_check') or {}).get('mismatches')}")
except Exception as e:
    print(v, "rc", rc, "no result", e)
PY
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
