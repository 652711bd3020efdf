#!/usr/bin/env bash
# C5 + verify counter evidence at HEAD: the SQ passes of tools/prof_pieces.sh, one
# FETCH_SIZE pass, and an LDS-unaligned-stall pass over bench.py (headline kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-r03sq}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
bash tools/prof_pieces.sh "$TAG" || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o c5 -- python3 "$ROOT/tools/prof_pieces.py" 3 > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/bench_lds" -o b -- python3 "$ROOT/bench.py" --steps 5 --warmup 5 --no-cpu-baseline --no-probe > "$OUT/bench_lds.log" 2>&1 || exit $?
echo done
