#!/bin/bash
# Profile each workload in $WORKLOADS with tools/gpu_profile.sh (kernel trace + separate PMC passes);
# results land in gpurun_out/<workload>_pmc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in ${WORKLOADS:-c3 c2}; do
  rm -rf gpurun_out/pmc_* gpurun_out/trace.log
  BENCH_ARGS="--workload $wl --steps 2 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit $?
  rm -rf "gpurun_out/${wl}_pmc" && mkdir -p "gpurun_out/${wl}_pmc"
  mv gpurun_out/pmc_* gpurun_out/trace.log "gpurun_out/${wl}_pmc/"
done
