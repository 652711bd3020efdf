#!/usr/bin/env python3
"""Why is a 2 M-packet (3 GB) shard slower per byte than 1 M (1.5 GB)?  Interleaved on
one box, 10 back-to-back calls per timing: the CRC kernel and the plain streaming-read
probe (libwtp_diag read_xor) over (a) the first 1.5 GB repeatedly, (b) alternating
halves, (c) the whole 3 GB per call.  If only the CRC kernel slows down with the
footprint, its access pattern (waves drifting apart: a wide active window) is the cause,
not the memory system's capacity for a cyclic stream."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent, diag  # noqa: E402

P = 1456
n = 2 << 20
h = n // 2
buf = torch.empty(n * P + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * P)
out = torch.empty(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
D = diag()


def crc(off, cnt):
    W.crc32_batch_fixed(buf[off * P:], P, P, cnt, out)


def probe(off, cnt):
    assert D.wtp_diag_read_xor(buf.data_ptr() + off * P, cnt * P, sink.data_ptr(), cus, 512, st.cuda_stream) == 0


V = {}
for name, f in (("crc", crc), ("probe", probe)):
    V[f"{name} 1st half x2"] = (lambda f=f: (f(0, h), f(0, h)), 2 * h)
    V[f"{name} halves alternate"] = (lambda f=f: (f(0, h), f(h, h)), 2 * h)
    V[f"{name} 2M"] = (lambda f=f: f(0, n), n)
for _ in range(60):
    for f, _c in V.values():
        f()
torch.cuda.synchronize()
res = {k: [] for k in V}
for rep in range(10):
    for k, (f, c) in V.items():
        a, b = TimingEvent(), TimingEvent()
        a.record(st)
        for _ in range(5):
            f()
        b.record(st)
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 5 / (c / h) * 1e3)
print(json.dumps({k: {"us_per_1M": round(float(np.median(v)), 1), "TBps": round(h * P / float(np.median(v)) / 1e6, 3)}
                  for k, v in res.items()}, indent=1))
