#!/usr/bin/env bash
# C4 per-rank step (2 M, one-rank RCCL gather every 2 steps) with 2 vs 8 result-slot groups, alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/${1:-groups}"; mkdir -p "$OUT"
for rep in 1 2 3; do
  for g in 2 8; do
    timeout -k 10 200 python bench.py --gather-n1 --packets-per-rank 2097152 --steps 40 --warmup 5 --no-cpu-baseline --no-probe \
      --result-groups $g > "$OUT/g${g}_r$rep.log" 2>&1 || exit $?
    python3 -c "import json,sys; l=[json.loads(x) for x in open('$OUT/g${g}_r$rep.log') if x.startswith('{')][-1]; print('g=$g rep=$rep', l['step_ms'], l['kernel_ms_max_over_ranks'], l['overlap'], l['per_rank_gather_ms'], l['parity']['match'])"
  done
done
