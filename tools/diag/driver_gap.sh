#!/bin/bash
# GPU box: the driver's exact bench command beside the long one, on one box,
# plus per-step event times of a short and a long run (FNNUE_STEP_EVENTS):
# is the driver's lower number warm-up, clock or box?
set -uo pipefail
D=gpurun_out/driver_gap
mkdir -p $D
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $D/$n.json 2> $D/$n.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads([l for l in open('$D/$n.json') if l.startswith('{')][-1])
st=d.get('step_ms'); r=d['roofline']
print('%-10s %8.1fM/s  ms/step %.4f  ft %.4f  %s' % ('$n', d['value']/1e6, d['ms_per_step'], r['kernel_avg_ms'],
      ('steps: first5 ' + ' '.join('%.3f' % x for x in st[:5]) + '  median %.3f' % sorted(st)[len(st)//2]) if st else ''))"
  return $rc
}
run driver1 --gpus 1 --steps 20 --warmup 5 && run driver2 --gpus 1 --steps 20 --warmup 5 && \
run long --steps 200 --no-cpu-baseline --no-host-api && \
FNNUE_STEP_EVENTS=1 run ev25 --steps 25 --warmup 5 --no-cpu-baseline --no-host-api && \
FNNUE_STEP_EVENTS=1 run ev200 --steps 200 --warmup 10 --no-cpu-baseline --no-host-api && \
run driver3 --gpus 1 --steps 20 --warmup 5
