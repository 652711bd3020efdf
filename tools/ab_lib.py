#!/usr/bin/env python3
"""Interleaved A/B of library builds in ONE process (each .so has its own device state):
   python tools/ab_lib.py --what build|crc|verify|c5 lib1.so lib2.so ...
Every round times each library's call back to back (timing-only events around 10
calls), so box drift hits all variants alike.  Prints the median us per call."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from bench import TimingEvent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="build")
ap.add_argument("--rounds", type=int, default=15)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()

vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
libs = []
for p in a.libs:
    L = C.CDLL(os.path.abspath(p))
    L.wtp_init.argtypes = [C.c_int]
    assert L.wtp_init(0) == 0
    L.wtp_build_data_packets.argtypes = [vp, sz, u32, vp, sz, vp, vp]
    L.wtp_crc32_batch_fixed.argtypes = [vp, sz, sz, sz, vp, vp]
    L.wtp_crc32_batch_var.argtypes = [vp, sz, vp, vp, sz, vp, vp]
    L.wtp_crc32_verify_batch.argtypes = [vp, sz, vp, sz, vp, vp, vp]
    L.wtp_synth_fill.argtypes = [vp, C.c_uint64, sz, C.c_uint64, vp]
    libs.append(L)
L0 = libs[0]
st = torch.cuda.current_stream()
sp = st.cuda_stream
n = a.n
P = 1456
if a.what in ("build", "crc", "verify", "crcalt", "verifyalt"):
    # crcalt / verifyalt: two n-packet batches (rings), the calls alternate between them (no
    # launch re-reads what the previous one read: a streaming sender / receiver)
    halves = 2 if a.what in ("crcalt", "verifyalt") else 1
    pay = torch.empty(halves * n * P + 64, dtype=torch.uint8, device="cuda")
    L0.wtp_synth_fill(pay.data_ptr(), 0, halves * n * P, 0x5EED, sp)
    ncall = [0]
    wire = torch.empty(n * 1472 + 64, dtype=torch.uint8, device="cuda")
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    L0.wtp_build_data_packets(pay.data_ptr(), n * P, 0, wire.data_ptr(), 1472, wl.data_ptr(), sp)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ref_wire = wire.clone()
    if a.what == "verifyalt":
        wire2 = torch.empty(n * 1472 + 64, dtype=torch.uint8, device="cuda")
        L0.wtp_build_data_packets(pay.data_ptr() + n * P, n * P, 0, wire2.data_ptr(), 1472, wl.data_ptr(), sp)
if a.what == "c5":
    lens = O.zipf_lengths(n, s=1.1)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    L0.wtp_synth_fill(d.data_ptr(), 0, total, 0x5EED, sp)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")


def call(L):
    if a.what == "build":
        L.wtp_build_data_packets(pay.data_ptr(), n * P, 0, wire.data_ptr(), 1472, wl.data_ptr(), sp)
    elif a.what == "crc":
        L.wtp_crc32_batch_fixed(pay.data_ptr(), P, P, n, out.data_ptr(), sp)
    elif a.what == "crcalt":
        ncall[0] += 1
        L.wtp_crc32_batch_fixed(pay.data_ptr() + (ncall[0] % 2) * n * P, P, P, n, out.data_ptr(), sp)
    elif a.what == "verify":
        L.wtp_crc32_verify_batch(wire.data_ptr(), 1472, wl.data_ptr(), n, ok.data_ptr(), None, sp)
    elif a.what == "verifyalt":
        ncall[0] += 1
        L.wtp_crc32_verify_batch((wire2 if ncall[0] % 2 else wire).data_ptr(), 1472, wl.data_ptr(), n, ok.data_ptr(),
                                 None, sp)
    elif a.what == "c5":
        L.wtp_crc32_batch_var(d.data_ptr(), total, do.data_ptr(), dl.data_ptr(), n, out.data_ptr(), sp)


for L in libs:
    for _ in range(30):
        call(L)
torch.cuda.synchronize()
res = {p: [] for p in a.libs}
checks = {}
for r in range(a.rounds):
    for p, L in zip(a.libs, libs):
        s, e = TimingEvent(), TimingEvent()
        s.record(st)
        for _ in range(10):
            call(L)
        e.record(st)
        torch.cuda.synchronize()
        res[p].append(s.elapsed_time(e) / 10 * 1e3)
        if r == 0 and a.what == "build":
            checks[p] = bool(torch.equal(wire, ref_wire))
        if r == 0 and a.what in ("crc", "crcalt"):
            if "want_crc" not in checks:
                checks["want_crc"] = out.clone()
            checks[p] = bool(torch.equal(out, checks["want_crc"]))
        if r == 0 and a.what == "c5":
            got = out.cpu().numpy().view(np.uint32)
            if "want" not in checks:
                checks["want"] = O.batch_var(d[:total].cpu().numpy(), offs, lens)
            checks[p] = bool(np.array_equal(got, checks["want"]))
checks.pop("want", None)
checks.pop("want_crc", None)
print(json.dumps({"what": a.what, "median_us": {os.path.basename(p): round(float(np.median(v)), 1) for p, v in res.items()},
                  "min_us": {os.path.basename(p): round(float(np.min(v)), 1) for p, v in res.items()},
                  "exact": {os.path.basename(p): v for p, v in checks.items()}}, indent=1))
