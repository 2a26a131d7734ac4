#!/bin/bash
# Profiling session: kernel trace + separate PMC passes (one counter group per run, no tracing
# domains mixed with --pmc).  Output under gpurun_out/pmc_*/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PROF_DIR:-.}
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
fatal() { [ "$1" -ge 124 ]; }
step() {
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc"; tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
}
BARGS=${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline}
# the build ids of the library this session profiles (tools/pmc_summary.py stamps its records with them)
python3 tools/kernel_ids.py > "$OUT/kernel_ids.json" || exit 1
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/pmc_trace -o run --output-format csv -- python3 bench.py $BARGS
# counter groups, ';'-separated (one rocprofv3 --pmc pass each)
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU;GRBM_GUI_ACTIVE GRBM_COUNT;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU_TRANS_F SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
IFS=';' read -r -a GROUPS_ARR <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  # shellcheck disable=SC2086
  step pmc_$i 300 rocprofv3 --pmc $grp -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py $BARGS
done
echo "profile session done"
