#!/usr/bin/env bash
# HBM read requests by size for the C5 and verify launches of tools/prof_pieces.py:
# pass 1 TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B, TCC_BUBBLE (128-B requests); pass 2 FETCH_SIZE.
# The verify launch reads a known byte count (1M x 1472-B ring) and calibrates the
# request-size formula; tools/tcc_bytes.py applies it to the C5 launch.  One rocprofv3
# --pmc pass per run, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-tcc}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for counters in "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_BUBBLE" "FETCH_SIZE"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o pp -- python3 "$ROOT/tools/prof_pieces.py" 3 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "  rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/p$i.log"; echo FATAL; exit $rc;; esac
done
echo done
