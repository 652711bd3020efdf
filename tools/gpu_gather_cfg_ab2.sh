#!/usr/bin/env bash
# C4 per-rank step (2 M, one-rank RCCL gather): gather grouping x result-slot groups, alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/${1:-gcfg2}"; mkdir -p "$OUT"
for rep in 1 2 3; do
  for cfg in "4 4" "4 2" "8 2" "8 4" "2 2"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --gather-n1 --packets-per-rank 2097152 --steps 40 --warmup 5 --no-cpu-baseline --no-probe \
      --gather-every $1 --result-groups $2 > "$OUT/e$1_g$2_r$rep.log" 2>&1 || exit $?
    python3 -c "import json; l=[json.loads(x) for x in open('$OUT/e$1_g$2_r$rep.log') if x.startswith('{')][-1]; print('every=$1 groups=$2 rep=$rep', l['step_ms'], l['roofline']['kernel_ms_mean'], l['kernel_ms_max_over_ranks'], l['overlap'], l['parity']['match'])"
  done
done
