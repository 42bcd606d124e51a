set -o pipefail
O=gpurun_out/${ROUND_TAG:-r02x}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
for wl in positions games children crazyhouse atomic; do
  a=""; [ $wl = children ] && a="--games 1000"
  timeout -k 10 240 python bench.py --workload $wl $a > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl rc=$?"; tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,1), d['ms_per_step'], d['roofline']['frac'], d['roofline']['bound'], d['roofline']['kernel_avg_ms'], d['roofline']['stack_kernel_avg_ms'], (d['cpu_baseline'] or {}).get('value'), d['parity_spot_check'])"
done
