set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbol.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sym_tests.log 2>&1; echo "sym tests rc=$?"; tail -1 gpurun_out/sym_tests.log
VARIANTS="default nowarm default nowarm" WORKLOADS="c3 c2" bash tools/ab.sh
