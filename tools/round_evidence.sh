#!/bin/bash
# GPU box: the round's evidence in one call — bench lines for the three
# workloads (with CPU baseline and host-API rate), then rocprofv3 kernel trace
# + PMC passes for configs 2 and 3.  Stops at the first failing step.
#   usage: tools/round_evidence.sh <tag>
tag=${1:-rXX}
mkdir -p gpurun_out
export PMCS="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE|TCC_HIT_sum TCC_MISS_sum"
step() { local name=$1; shift; "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 2 gpurun_out/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step bench_positions timeout -k 10 300 python bench.py
step bench_games timeout -k 10 300 python bench.py --workload games
step bench_children timeout -k 10 300 python bench.py --workload children --games 1000
step profile_positions timeout -k 10 900 tools/profile.sh ${tag}
step profile_games timeout -k 10 900 tools/profile.sh ${tag}_games --workload games
