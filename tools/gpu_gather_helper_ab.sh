#!/usr/bin/env bash
# C4 per-rank step (2 M, one-rank RCCL gather every 2 steps): torch's stream coupling vs a helper stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/${1:-ghelper}"; mkdir -p "$OUT"
for rep in 1 2 3; do
  for h in "" "--gather-helper"; do
    tag=$([ -n "$h" ] && echo helper || echo torch)
    timeout -k 10 200 python bench.py --gather-n1 --packets-per-rank 2097152 --steps 40 --warmup 5 --no-cpu-baseline --no-probe \
      $h > "$OUT/${tag}_r$rep.log" 2>&1 || exit $?
    python3 -c "import json; l=[json.loads(x) for x in open('$OUT/${tag}_r$rep.log') if x.startswith('{')][-1]; print('$tag rep=$rep', l['step_ms'], l['roofline']['kernel_ms_mean'], l['kernel_ms_max_over_ranks'], l['overlap'], l['per_rank_gather_ms'], l['parity']['match'])"
  done
done
