#!/usr/bin/env bash
# SQ counter passes (one rocprofv3 --pmc run each, kernel trace only) over the C5 /
# verify driver (tools/prof_pieces.py) for each library given (WTP_LIB A/B builds, or
# 'product'); output under
# gpurun_out/<tag>/<path>/.      usage: tools/prof_sq.sh <tag> <path>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-sq}"; shift; export TMPDIR=/tmp
for P in "$@"; do
  OUT="$ROOT/gpurun_out/$TAG/$P"; mkdir -p "$OUT"
  if [ "$P" != product ]; then export WTP_LIB="$ROOT/$P"; else unset WTP_LIB; fi
  i=0
  while read -r counters; do
    [ -z "$counters" ] && continue
    i=$((i+1))
    cd /tmp
    timeout -k 10 120 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o pp -- python3 "$ROOT/tools/prof_pieces.py" 3 > "$OUT/p$i.log" 2>&1
    rc=$?; echo "[$P pass $i] rc=$rc"
    case $rc in 0) ;; *) tail -5 "$OUT/p$i.log"; echo FATAL; exit $rc;; esac
  done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES
GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM
LIST
done
echo done
