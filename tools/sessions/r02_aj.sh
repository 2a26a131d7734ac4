set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbol.py tests/test_gpu_dist.py tests/test_bench_plan.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sym_tests.log 2>&1; rc=$?; echo "sym tests rc=$rc"; tail -3 gpurun_out/sym_tests.log
[ $rc -ge 2 ] && exit $rc
for v in default static nosplit default static nosplit; do
  if [ $v = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  for w in c2 c3; do
    echo -n "$v $w "; timeout -k 10 120 python bench.py --workload $w --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.4g' % d['value'], round(d['roofline']['avg_launch_ms'],4))" || exit 3
  done
done
