#!/usr/bin/env bash
# Kernel trace of k_stream just below and just above a 2 GiB buffer (tools/stream_2g_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; OUT="$ROOT/gpurun_out/${1:-s2gt}"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for n in 15800000 15900000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n$n" -o s -- python3 "$ROOT/tools/stream_2g_probe.py" $n 5 > "$OUT/n$n.log" 2>&1
  rc=$?; echo "n=$n rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/n$n.log"; exit $rc;; esac
done
echo done
