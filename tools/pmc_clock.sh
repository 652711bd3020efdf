#!/usr/bin/env bash
# Effective clock and instruction counts per braided-kernel variant (diagnostic):
# GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md, DVFS give-back), one PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-clk}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
KB_ONLY="${KB_ONLY:-braid_nolut,braid_skel}" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv \
  -d "$OUT/pmc" -o kb -- "$ROOT/tools/bin/kbench" 1048576 10 > "$OUT/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
