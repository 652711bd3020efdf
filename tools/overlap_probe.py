#!/usr/bin/env python3
"""Can a small kernel on a second stream run beside the persistent CRC kernel?  Models
bench.py's pipelined N>1 step on one GPU: stream A runs the 1 M x 1456 CRC launches;
after each, stream B waits for it and copies the 4 MiB of results (standing in for the
RCCL gather's kernel), while A goes straight on to the next CRC.  Reports per-step time
for CRC alone, CRC + copy serialised on A, and the two-stream pipeline, each with 0 and
8 reserved CUs.
  python tools/overlap_probe.py [--steps 50]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=50)
a = ap.parse_args()
n = 1 << 20
buf = torch.empty(n * 1456 + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * 1456)
outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
dst = torch.empty(8 * n, dtype=torch.int32, device="cuda")  # "gathered" (8 ranks' worth)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def run(mode, steps):
    done = [torch.cuda.Event() for _ in range(steps)]
    copied = [torch.cuda.Event() for _ in range(steps)]
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0.record(sa)
    for i in range(steps):
        o = outs[i % 2]
        if mode == "pipe" and i >= 2:
            sa.wait_event(copied[i - 2])
        W.crc32_batch_fixed(buf, 1456, 1456, n, o, sa)
        if mode == "serial":
            with torch.cuda.stream(sa):
                dst[:n].copy_(o)
        elif mode == "pipe":
            done[i].record(sa)
            sb.wait_event(done[i])
            with torch.cuda.stream(sb):
                dst[(i % 8) * n:(i % 8 + 1) * n].copy_(o)
            copied[i].record(sb)
    if mode == "pipe":
        sa.wait_stream(sb)
    t1.record(sa)
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / steps


for _ in range(200):
    W.crc32_batch_fixed(buf, 1456, 1456, n, outs[0], sa)
torch.cuda.synchronize()
for rep in range(3):
    for r in (0, 8):
        W.reserve_cus(r)
        res = {m: run(m, a.steps) for m in ("crc", "serial", "pipe")}
        print(f"rep {rep} reserve {r}: us/step crc-only {res['crc']:.1f}  crc+copy serial {res['serial']:.1f}  "
              f"two-stream pipeline {res['pipe']:.1f}", flush=True)
W.reserve_cus(0)
