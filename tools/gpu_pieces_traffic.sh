#!/usr/bin/env bash
# FETCH_SIZE of the general kernel's three traffic-attribution batches (tools/prof_pieces_traffic.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; OUT="$ROOT/gpurun_out/${1:-ptraffic}"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/p1" -o pt -- python3 "$ROOT/tools/prof_pieces_traffic.py" 3 > "$OUT/p1.log" 2>&1
echo "rc=$?"
