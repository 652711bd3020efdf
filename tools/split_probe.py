#!/usr/bin/env python3
"""Is C4's 2 M-packet shard slower per byte than the 1 M headline batch because of the
launch length?  Interleaved, on one box: one 2 M launch vs the same 2 M packets as
2 x 1 M, 4 x 512 K and 8 x 256 K launches back to back (timing-only events around each
step), and the 1 M batch alone.  Prints median / mean us per step and TB/s."""
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
n = 2 << 20
buf = torch.empty(n * P + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * P)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()


def step(parts):
    per = n // parts
    for k in range(parts):
        W.crc32_batch_fixed(buf[k * per * P:], P, P, per, out[k * per:])


variants = {"2M x1": lambda: step(1), "1M x2": lambda: step(2), "512K x4": lambda: step(4), "256K x8": lambda: step(8),
            "1M alone": lambda: W.crc32_batch_fixed(buf, P, P, n // 2, out),
            "1M second half": lambda: W.crc32_batch_fixed(buf[(n // 2) * P:], P, P, n // 2, out)}
for _ in range(150):
    step(1)
torch.cuda.synchronize()
res = {k: [] for k in variants}
for rep in range(12):
    for k, f in variants.items():
        a, b = TimingEvent(), TimingEvent()
        a.record(st)
        for _ in range(10):
            f()
        b.record(st)
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 10 * 1e3)
summary = {}
for k, v in res.items():
    byts = (n // 2 if k.startswith("1M ") else n) * P
    med = float(np.median(v))
    summary[k] = {"median_us": round(med, 1), "mean_us": round(float(np.mean(v)), 1), "TBps": round(byts / med / 1e6, 3)}
print(json.dumps(summary, indent=1))
