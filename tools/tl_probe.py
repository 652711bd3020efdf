#!/usr/bin/env python3
"""Address-translation counters for DESIGN 7.11 (why a 2 M shard, or a launch over other
memory than the previous one, is ~5% slower per byte than re-reading one 1 M buffer).

One process, fixed dispatch order, so a rocprofv3 --pmc pass can be split by phase:
  crc  x WARM   warmup over the first 1 M packets (1.5 GB)
  crc  x K      "repeat":    the same first half every launch
  crc  x K      "alternate": first half, second half, first half, ...
  crc  x K      "2M":        one launch over both halves (3.05 GB)
  probe x WARM, probe x K repeat, probe x K alternate   (libwtp_diag read_xor)
Without a profiler it prints the HIP-event time per phase; tools/tl_summary.py splits a
counter CSV by the same order.

    tl_probe.py [--k 10] [--warm 20] [--out phases.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent, diag  # noqa: E402

P = 1456
ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--warm", type=int, default=20)
ap.add_argument("--out", default=None)
a = ap.parse_args()

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


phases = []


def phase(name, kernel, fn, k, per_launch_packets):
    ev = [(TimingEvent(), TimingEvent()) for _ in range(k)]
    for i in range(k):
        ev[i][0].record(st)
        fn(i)
        ev[i][1].record(st)
    torch.cuda.synchronize()
    us = [s.elapsed_time(e) * 1e3 for s, e in ev]
    phases.append({"phase": name, "kernel": kernel, "launches": k, "packets_per_launch": per_launch_packets,
                   "median_us": round(sorted(us)[k // 2], 1),
                   "median_us_per_1M": round(sorted(us)[k // 2] * h / per_launch_packets, 1)})


torch.cuda.synchronize()
phase("crc warm", "crc", lambda i: crc(0, h), a.warm, h)
phase("crc repeat", "crc", lambda i: crc(0, h), a.k, h)
phase("crc alternate", "crc", lambda i: crc(h * (i % 2), h), a.k, h)
phase("crc 2M", "crc", lambda i: crc(0, n), a.k, n)
phase("probe warm", "probe", lambda i: probe(0, h), a.warm, h)
phase("probe repeat", "probe", lambda i: probe(0, h), a.k, h)
phase("probe alternate", "probe", lambda i: probe(h * (i % 2), h), a.k, h)
res = {"order": phases, "note": "dispatch order per kernel: crc phases then probe phases, as listed"}
print(json.dumps(res, indent=1))
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
