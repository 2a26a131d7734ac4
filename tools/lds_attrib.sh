#!/bin/bash
# LDS conflict attribution of frame_sync_kernel: one PMC pass (SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE,
# SQ_WAVES) of the frame bench per variant library (default + the FRAME_DUP_<SITE> probes, tools/build_variants.py);
# tools/lds_attrib.py turns the deltas into per-site instruction / conflict / array-cycle counts per item.
# The probes were pruned from csrc/ in round 6: their libraries are built from commit aec0f2e (profiles/r06/README.md).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/${PROF_DIR:-lds_attrib}
mkdir -p "$OUT"
for v in ${VARIANTS:-default dupdet dupmf dupcap dupbp dupcfo}; do
  if [ "$v" = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d "$OUT/$v" -o run \
    --output-format csv -- python3 bench.py --workload ${WORKLOAD:-frame} --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/$v.log"; exit $rc; }
done
exit 0
