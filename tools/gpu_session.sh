#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && step smoke 400 python3 -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && step gpu_tests 1200 python3 -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && step bench 600 python3 bench.py ${BENCH_ARGS:-}
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo "session done"
