#!/usr/bin/env bash
# Ablation timings + PMC counters for the braided kernel (diagnostic session).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-kb}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { local name="$1" secs="$2"; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "  rc=$rc"; tail -n 12 "$OUT/$name.log"; case $rc in 0|1) ;; *) echo FATAL; exit $rc;; esac; }
step kbench 300 "$ROOT/tools/bin/kbench" 1048576 20
cd /tmp
step listpmc 120 rocprofv3 -L
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o kb -- "$ROOT/tools/bin/kbench" 1048576 2
step pmc_sq 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o kb -- "$ROOT/tools/bin/kbench" 1048576 2
echo done
