#!/bin/bash
# GPU box: kernel-trace A/B of replay builds (tools/exp_build.sh): median
# replay kernel time per batch count for each library.
#   usage: tools/diag/replay_ab.sh name1 name2 ...   ("main" = fishnet_amd/libfnnue.so)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/replay_ab
for v in "$@"; do
  lib=$PWD/exp/libfnnue_$v.so; [ $v = main ] && lib=$PWD/fishnet_amd/libfnnue.so
  out=gpurun_out/replay_ab/$v
  FNNUE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out -o run -- \
    python3 bench.py --workload backend --go-batches ${SIZES:-1,64,1024,16384} --go-calls 30 --warmup 2 --no-cpu-baseline \
    > $out.json 2> $out.log
  rc=$?
  [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $out.log; exit $rc; }
  python3 tools/diag/replay_summary.py $v $out
done
