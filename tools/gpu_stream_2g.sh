#!/usr/bin/env bash
# Counter passes of k_stream just below and just above a 2 GiB buffer (tools/stream_2g_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; OUT="$ROOT/gpurun_out/${1:-s2g}"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for n in 15800000 15900000; do
  i=0
  for counters in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY" "FETCH_SIZE" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d "$OUT/n${n}_p$i" -o s -- python3 "$ROOT/tools/stream_2g_probe.py" $n 3 > "$OUT/n${n}_p$i.log" 2>&1
    rc=$?; echo "n=$n pass $i rc=$rc"
    case $rc in 0) ;; *) tail -5 "$OUT/n${n}_p$i.log"; exit $rc;; esac
  done
done
echo done
