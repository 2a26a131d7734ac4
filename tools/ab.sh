#!/bin/bash
# A/B bench of variant libraries (tools/build_variants.py) on the GPU box.
# usage: VARIANTS="default nofence" WORKLOADS="c3 c2" bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  for wl in ${WORKLOADS:-c3}; do
    if [ "$v" = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
    timeout -k 10 200 python3 bench.py --workload "$wl" --symbols "${SYMBOLS:-10000000}" --no-cpu-baseline \
      > "gpurun_out/ab_${wl}_$v.json" 2> "gpurun_out/ab_${wl}_$v.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc for $v $wl"; tail -5 "gpurun_out/ab_${wl}_$v.err"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4g' % d['value'], round(d['roofline']['avg_launch_ms'], 3))" "gpurun_out/ab_${wl}_$v.json" "$v" "$wl"
  done
done
