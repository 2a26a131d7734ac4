#!/bin/bash
# Run a list of GPU steps on the box, each under its own time limit; a test failure (rc 1) does not
# stop the list, a fault / abort / timeout (rc >= 2 except pytest's 1) ends it at once.
# usage: bash tools/gpu_steps.sh STEPFILE      (lines: NAME SECONDS COMMAND...; '#' comments)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
while read -r name secs cmd; do
  [[ -z "${name:-}" || "$name" == \#* ]] && continue
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] end $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ "$rc" -ge 2 ]; then echo "fatal rc=$rc in $name: stopping"; exit "$rc"; fi
done < "$1"
echo "steps done"
