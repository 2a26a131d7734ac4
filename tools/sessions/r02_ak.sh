set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbol.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sym_tests.log 2>&1; rc=$?; echo "sym tests rc=$rc"; tail -3 gpurun_out/sym_tests.log
[ $rc -ge 2 ] && exit $rc
for v in default static default static; do
  if [ $v = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  echo -n "$v c5 "; timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.4g' % d['value'], round(d['roofline']['avg_launch_ms'],4))" || exit 3
done
