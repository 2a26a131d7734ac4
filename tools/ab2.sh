#!/bin/bash
# Interleaved A/B bench of variant libraries (tools/build_variants.py) on the GPU box: REPS rounds of
# (every variant x every workload), so box drift hits all variants alike.  Default workload sizes.
# usage: VARIANTS="default lswf" WORKLOADS="c3 c2" REPS=3 bash tools/ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in $(seq 1 "${REPS:-2}"); do
  for wl in ${WORKLOADS:-c3}; do
    case $wl in c2) args="--steps 60 --warmup 10";; frame*) args="--steps 4 --warmup 1";; *) args="--steps 10 --warmup 3";; esac
    for v in ${VARIANTS:-default}; do
      if [ "$v" = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
      out=gpurun_out/ab/${wl}_${v}_$r.json
      timeout -k 10 200 python3 bench.py --workload "$wl" $args --no-cpu-baseline ${BENCH_EXTRA:-} > "$out" 2> "${out%.json}.err"
      rc=$?
      if [ $rc -ne 0 ]; then echo "rc=$rc for $v $wl"; tail -5 "${out%.json}.err"; exit $rc; fi
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], '%.5g' % d['value'], round(d['roofline']['avg_launch_ms'], 4))" "$out" "$r" "$wl" "$v"
    done
  done
done
