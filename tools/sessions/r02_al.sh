# closing checkpoint: full GPU suite, smoke, bench lines, kernel-trace stats of the default bench
set -u
mkdir -p gpurun_out/closing2
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/closing2/gpu_tests.txt 2>&1 || { tail -20 gpurun_out/closing2/gpu_tests.txt; exit 3; }
tail -2 gpurun_out/closing2/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/closing2/smoke.txt 2>&1 || { tail -20 gpurun_out/closing2/smoke.txt; exit 3; }
cat gpurun_out/closing2/smoke.txt | tail -1
timeout -k 10 400 python bench.py > gpurun_out/closing2/bench_default.json 2> gpurun_out/closing2/bench_default.err || exit 3
tail -1 gpurun_out/closing2/bench_default.json
for wl in c2 c4 c5 frame; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/closing2/bench_$wl.json 2> gpurun_out/closing2/bench_$wl.err || exit 3
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], round(d['roofline']['avg_launch_ms'],4))" gpurun_out/closing2/bench_$wl.json $wl
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/closing2/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/closing2/trace.log 2>&1 || exit 3
tail -1 $GRAFT_REPO_ROOT/gpurun_out/closing2/trace.log
