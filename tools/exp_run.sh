#!/bin/bash
# GPU box: A/B of experimental builds (tools/exp_build.sh) against the main
# library, alternating so box drift hits every variant alike.
#   usage: WLS="positions games" ROUNDS=2 tools/exp_run.sh name1 name2 ...
# "main" names fishnet_amd/libfnnue.so.  Extra bench args in $BENCH_ARGS.
mkdir -p gpurun_out/exp
WLS=${WLS:-positions}
for r in $(seq 1 ${ROUNDS:-2}); do
  for wl in $WLS; do
    for v in main "$@"; do
      lib=$PWD/exp/libfnnue_$v.so; [ $v = main ] && lib=$PWD/fishnet_amd/libfnnue.so
      log=gpurun_out/exp/${v}_${wl}_$r.log
      FNNUE_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-100} --cpu-seconds 1 \
        --no-host-api ${BENCH_ARGS:-} > $log 2>&1
      rc=$?
      python3 - "$v" "$wl" "$rc" "$log" <<'PY'
import json, sys
v, wl, rc, log = sys.argv[1:5]
try:
    d = json.loads([l for l in open(log) if l.startswith("{")][-1])
    r = d["roofline"]
    print(f"{v:10s} {wl:9s} {d['value']/1e6:8.1f}M/s plan={r['plan_avg_ms']:.4f} ft={r['kernel_avg_ms']:.4f} "
          f"stack={r['stack_kernel_avg_ms']:.4f} mism={(d.get('parity_spot_check') or {}).get('mismatches')}", flush=True)
except Exception as e:
    print(v, wl, "rc", rc, "no result", e, flush=True)
PY
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; tail -5 $log; exit $rc; fi
    done
  done
done
