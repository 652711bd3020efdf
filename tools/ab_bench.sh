#!/usr/bin/env bash
# A/B the headline kernel: bench.py with each library in a3-reliable-transport_amd/lib/ab/,
# interleaved twice (A B A B) to average out box drift, plus one FETCH_SIZE pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"; TAG="${1:-abb}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in a3-reliable-transport_amd/lib/ab/*.so; do
    v=$(basename "$lib" .so)
    WTP_LIB="$ROOT/$lib" timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_${v}_$rep.log" 2>&1
    rc=$?; echo "$v rep$rep rc=$rc $(grep -o '"kernel_ms_mean": [0-9.]*' "$OUT/bench_${v}_$rep.log")"
    case $rc in 0) ;; *) echo FATAL; exit $rc;; esac
  done
done
cd /tmp
for lib in "$ROOT"/a3-reliable-transport_amd/lib/ab/*.so; do
  v=$(basename "$lib" .so)
  WTP_LIB="$lib" timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$v" -o b -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/pmc_$v.log" 2>&1
  rc=$?; echo "pmc $v rc=$rc"; case $rc in 0) ;; *) echo FATAL; exit $rc;; esac
done
echo done
