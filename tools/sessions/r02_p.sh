set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_message.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/frame_tests.log 2>&1; echo "frame tests rc=$?"; tail -2 gpurun_out/frame_tests.log
OFDM_MI355X_LIB=variants/libofdm_k1wave.so timeout -k 10 200 python -u -m pytest tests/test_gpu_symbol.py -x -q -k fft --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/k1wave_tests.log 2>&1; echo "k1wave tests rc=$?"; tail -2 gpurun_out/k1wave_tests.log
timeout -k 10 120 python tools/fft_ab.py > gpurun_out/fft_default.json 2>gpurun_out/fft_default.err; echo "fft default rc=$?"; cat gpurun_out/fft_default.json
OFDM_MI355X_LIB=variants/libofdm_k1wave.so timeout -k 10 120 python tools/fft_ab.py > gpurun_out/fft_k1wave.json 2>gpurun_out/fft_k1wave.err; echo "fft k1wave rc=$?"; cat gpurun_out/fft_k1wave.json
SYMBOLS=1000000 VARIANTS="default wfull default wfull" WORKLOADS="frame" bash tools/ab.sh
