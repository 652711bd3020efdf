#!/usr/bin/env python3
"""Is one 2 M-packet braided launch slower than the same packets in 2 or 4 launches?
C4's per-rank shard (2 M x 1456 B) timed per step (events around the step's launches),
interleaved: 1 x 2 M, 2 x 1 M, 4 x 512 K, 3 x 699,051 (+1), 20 rounds of 10 steps.
Also the 1 M headline launch alone for reference.  Diagnostic."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent  # noqa: E402

P = 1456
n = 2 * 1048576
assert W.LIB.wtp_init(0) == 0
buf = torch.empty(n * P + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * P)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()


def step(k):
    per = [n * i // k for i in range(k + 1)]
    for a, b in zip(per, per[1:]):
        W.crc32_batch_fixed(buf[a * P:], P, P, b - a, out[a:], st)


variants = {"1x2M": 1, "2x1M": 2, "3x": 3, "4x512K": 4}
ref = None
res = {k: [] for k in variants}
for k, v in variants.items():
    for _ in range(20):
        step(v)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(out, ref), k
for r in range(20):
    for k, v in variants.items():
        s, e = TimingEvent(), TimingEvent()
        s.record(st)
        for _ in range(10):
            step(v)
        e.record(st)
        torch.cuda.synchronize()
        res[k].append(s.elapsed_time(e) / 10)
print(json.dumps({"ms_per_step_median": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                  "ms_per_step_min": {k: round(float(np.min(v)), 4) for k, v in res.items()}}, indent=1))
