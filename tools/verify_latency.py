#!/usr/bin/env python3
"""Per-call latency of small receiver-verify batches (wReceiver's regime): the device
entry point (braided pass + fix-up pass) against a single braided CRC launch of the same
payloads, and the host wrapper from a pinned ring (H2D, verify, D2H).
  python tools/verify_latency.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

stride = 1504
for n in (64, 1024, 16384):
    pay = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(pay)
    wire = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    W.build_data_packets(pay, n * 1456, 0, wire, stride, wl)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    out = torch.zeros(n, dtype=torch.int32, device="cuda")

    def t_dev(f, reps=200):
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return float(np.median(ts))

    v = t_dev(lambda: W.verify_batch(wire, stride, wl, n, ok))
    c = t_dev(lambda: W.crc32_batch_fixed(pay, 1456, 1456, n, out))
    ring = W.PinnedBuffer(n * stride) if hasattr(W, "PinnedBuffer") else None
    host = wire.cpu().numpy()
    rl = wl.cpu().numpy().view(np.uint32)
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        okh, crch = W.host_verify(host, stride, rl)
        ts.append((time.perf_counter() - t0) * 1e6)
    assert okh.all()
    print(f"n={n}: device verify {v:.1f} us (braided + fix-up pass) vs one CRC launch {c:.1f} us; "
          f"host_verify (pageable numpy ring) median {np.median(ts):.1f} us", flush=True)
