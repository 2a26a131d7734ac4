# round 5: lazy long-capture kernel -- frame/message GPU tests, then frame8 with the lazy round-2 skip
# (default) against every capture in full (OFDM_FRAME_NO_LAZY=1), interleaved
set -u
mkdir -p gpurun_out/lazy8
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame.py tests/test_gpu_message.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/lazy8/tests.txt 2>&1 || { tail -30 gpurun_out/lazy8/tests.txt; exit 1; }
tail -2 gpurun_out/lazy8/tests.txt
for r in 1 2 3; do
  for v in full lazy; do
    if [ $v = full ]; then export OFDM_FRAME_NO_LAZY=1; else unset OFDM_FRAME_NO_LAZY; fi
    timeout -k 10 200 python3 bench.py --workload frame8 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/lazy8/f8_${v}_$r.json 2> gpurun_out/lazy8/f8_${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.5g' % d['value'], round(d['roofline']['avg_launch_ms'],4))" gpurun_out/lazy8/f8_${v}_$r.json $r $v
  done
done
