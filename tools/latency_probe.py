#!/usr/bin/env python3
"""Where a window-size host verify call spends its time: launch + sync of an empty
kernel, the device verify of 10 datagrams (+ sync), and wtp_crc32_host_verify from a
pinned ring (zero copy), medians over 2000 calls.   python tools/latency_probe.py"""
import ctypes as C
import json
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


def med(fn, reps=2000):
    for _ in range(50):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 2)


res = {}
x = torch.zeros(1, device="cuda")
res["empty_kernel_plus_sync_us"] = med(lambda: (x.add_(1), torch.cuda.synchronize()))
res["sync_only_us"] = med(torch.cuda.synchronize)
hip = C.CDLL("libamdhip64.so")
res["hipDeviceSynchronize_only_us"] = med(lambda: hip.hipDeviceSynchronize())
n, stride = 10, 1504
pay = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
W.synth_fill(pay)
wire = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
wl = torch.empty(n, dtype=torch.int32, device="cuda")
W.build_data_packets(pay, n * 1456, 0, wire, stride, wl)
ok = torch.empty(n, dtype=torch.uint8, device="cuda")
res["device_verify_10_plus_sync_us"] = med(lambda: (W.verify_batch(wire, stride, wl, n, ok), torch.cuda.synchronize()))
ring = W.PinnedBuffer(n * stride)
ring.array[:] = wire.cpu().numpy()
lens = W.PinnedBuffer(n * 4)
la = lens.array.view(np.uint32)
la[:] = wl.cpu().numpy().view(np.uint32)
res["host_verify_10_zero_copy_us"] = med(lambda: W.host_verify(ring.array, stride, la))
okh, _ = W.host_verify(ring.array, stride, la)
res["all_ok"] = bool(okh.all())
print(json.dumps(res))
