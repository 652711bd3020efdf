#!/usr/bin/env python3
"""What do bench.py's per-launch timing events cost the step?  The headline kernel (1 M x
1456 B) launched 20 times back to back, interleaved rounds of: (a) start+end event per
launch (bench.py's timed loop), (b) one end event per launch, (c) events around the 20
launches only.  Per-step time from the region events, and host wall time.  Diagnostic."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent  # noqa: E402

P, N, K = 1456, 1 << 20, 20
assert W.LIB.wtp_init(0) == 0
buf = torch.empty(N * P + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=N * P)
out = torch.empty(N, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
for _ in range(50):
    W.crc32_batch_fixed(buf, P, P, N, out, st)
torch.cuda.synchronize()
res = {"per_launch_pair": [], "per_launch_end": [], "region_only": []}
wall = {k: [] for k in res}
for r in range(12):
    for mode in res:
        evs = [(TimingEvent(), TimingEvent()) for _ in range(K)]
        a, b = TimingEvent(), TimingEvent()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(st)
        for i in range(K):
            if mode == "per_launch_pair":
                evs[i][0].record(st)
            W.crc32_batch_fixed(buf, P, P, N, out, st)
            if mode != "region_only":
                evs[i][1].record(st)
        b.record(st)
        torch.cuda.synchronize()
        wall[mode].append((time.perf_counter() - t0) / K * 1e3)
        res[mode].append(a.elapsed_time(b) / K)
print(json.dumps({"ms_per_step_median": {k: round(float(np.median(v)), 5) for k, v in res.items()},
                  "wall_ms_per_step_median": {k: round(float(np.median(v)), 5) for k, v in wall.items()}}, indent=1))
