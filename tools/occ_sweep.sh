set -u
cd "${GRAFT_REPO_ROOT}"
export OFDM_MI355X_LIB=variants/libofdm_grid.so
for b in 1 2 3; do
  OFDM_RX_BLOCKS_PER_CU=$b timeout -k 10 120 python3 bench.py --workload c3 --symbols 4000000 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/occ_$b.json 2> gpurun_out/occ_$b.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], round(d['roofline']['avg_launch_ms'], 3))" gpurun_out/occ_$b.json $b
done
