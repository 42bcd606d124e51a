set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_dec2.log 2>&1 || { tail -30 gpurun_out/gputest_dec2.log; exit 1; }
tail -1 gpurun_out/gputest_dec2.log
WLS="games children crazyhouse-games" ROUNDS=2 bash tools/exp_run.sh sd || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr3_games -o run -- python3 bench.py --workload games --steps 10 --warmup 2 --no-cpu-baseline --no-host-api > gpurun_out/tr3_games.log 2>&1 || exit 1
echo done
