set -u
mkdir -p gpurun_out
for v in k1w8 k1w16; do
OFDM_MI355X_LIB=variants/libofdm_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_symbol.py -x -q -k fft --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${v}_tests.log 2>&1; echo "$v tests rc=$?"; tail -1 gpurun_out/${v}_tests.log
done
for v in default k1w8 k1w16; do
  if [ $v = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  timeout -k 10 120 python tools/fft_ab.py > gpurun_out/fft_$v.json 2>gpurun_out/fft_$v.err; echo "$v rc=$?"; cat gpurun_out/fft_$v.json
done
