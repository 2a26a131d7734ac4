set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_message.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/frame_tests.log 2>&1; rc=$?; echo "frame tests rc=$rc"; tail -3 gpurun_out/frame_tests.log
[ $rc -ge 2 ] && exit $rc
SYMBOLS=1000000 VARIANTS="default row default row" WORKLOADS="frame" bash tools/ab.sh
