#!/usr/bin/env python3
"""Interleaved A/B of the braided kernel's grid: all CUs vs CUs left free with
wtp_reserve_cus (1 M x 1456 B, same process, alternating blocks of launches).
  python tools/ab_reserve.py [--reserve 0,8,16] [--reps 6] [--launches 100]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reserve", default="0,8,16")
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--launches", type=int, default=100)
ap.add_argument("--n", type=int, default=1 << 20)
a = ap.parse_args()
res = [int(x) for x in a.reserve.split(",")]
n = a.n
buf = torch.empty(n * 1456 + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * 1456)
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
times = {r: [] for r in res}
for _ in range(300):  # past the clock transient
    W.crc32_batch_fixed(buf, 1456, 1456, n, out)
torch.cuda.synchronize()
for rep in range(a.reps):
    for r in res:
        W.reserve_cus(r)
        for _ in range(5):
            W.crc32_batch_fixed(buf, 1456, 1456, n, out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches + 1)]
        ev[0].record()
        for i in range(a.launches):
            W.crc32_batch_fixed(buf, 1456, 1456, n, out)
            ev[i + 1].record()
        torch.cuda.synchronize()
        ts = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.launches)]
        times[r].append(float(np.median(ts)))
        got = out.cpu().numpy()
        if ref is None:
            ref = got.copy()
        assert np.array_equal(got, ref), r
W.reserve_cus(0)
for r in res:
    t = times[r]
    print(f"reserve {r:3d}: median-of-medians {np.median(t):7.2f} us  reps {[round(x, 1) for x in t]}  "
          f"{n * 1456 / (np.median(t) * 1e-6) / 8e12:.4f} of 8 TB/s", flush=True)
