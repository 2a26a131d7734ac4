set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_bench_plan.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/plan_tests.log 2>&1; rc=$?; echo "plan tests rc=$rc"; tail -3 gpurun_out/plan_tests.log
[ $rc -ne 0 ] && exit 3
for v in 1 0 1 0; do
  for wl in c3 c4; do
    echo -n "prefetch=$v $wl "; OFDM_BENCH_TX_PREFETCH=$v timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.4g' % d['value'], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],4))" || exit 3
  done
done
