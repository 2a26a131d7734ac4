set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbol.py -k fft -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fft_tests.log 2>&1; rc=$?; echo "fft tests rc=$rc"; tail -3 gpurun_out/fft_tests.log
[ $rc -ge 2 ] && exit $rc
for v in default quad1 quad4 wave default; do
  if [ $v = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  echo -n "$v "; timeout -k 10 120 python tools/fft_ab.py 2>/dev/null || exit 3
done
