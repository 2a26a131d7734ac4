set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_message.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/frame_tests.log 2>&1; echo "frame tests rc=$?"; tail -1 gpurun_out/frame_tests.log
OFDM_MI355X_LIB=variants/libofdm_t256w4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/frame_tests_t256.log 2>&1; echo "frame tests t256w4 rc=$?"; tail -1 gpurun_out/frame_tests_t256.log
SYMBOLS=1000000 VARIANTS="default hoist t256w4 t256w5 t256w6 default" WORKLOADS="frame" bash tools/ab.sh
