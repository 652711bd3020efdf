#!/usr/bin/env python3
"""Does the allocation's page layout move the braided kernel's streaming rate?  The
UTCL1 misses of DESIGN 7.10 appear when a launch covers more memory than the CUs'
translations hold (two 1 M buffers alternately; one 2 M launch).  Same kernel, buffers
from torch (hipMalloc) vs hipExtMallocWithFlags(hipDeviceMallocContiguous), interleaved:
1 M same buffer, 1 M alternating between two buffers, one 2 M launch.  Diagnostic."""
import ctypes as C
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

P, N = 1456, 1 << 20
assert W.LIB.wtp_init(0) == 0
hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipExtMallocWithFlags.restype = C.c_int
st = torch.cuda.current_stream()
sp = st.cuda_stream
nb = 2 * N * P + 4096


def alloc(kind):
    if kind == "torch":
        t = torch.empty(nb, dtype=torch.uint8, device="cuda")
        return t, t.data_ptr()
    p = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(p), nb, {"contiguous": 4, "default_ext": 0}[kind])
    if rc != 0:
        return None, None
    return p, p.value


bufs = {}
for kind in ("torch", "contiguous", "default_ext"):
    keep, ptr = alloc(kind)
    if ptr is None:
        print(kind, "allocation failed", flush=True)
        continue
    base = (ptr + 255) & ~255
    W.LIB.wtp_synth_fill(base, 0, 2 * N * P, 0x5EED, sp)
    bufs[kind] = (keep, base)
torch.cuda.synchronize()
out = torch.empty(2 * N, dtype=torch.int32, device="cuda")
op = out.data_ptr()


def run(base, mode, i):
    if mode == "same":
        W.LIB.wtp_crc32_batch_fixed(base, P, P, N, op, sp)
    elif mode == "alt":
        W.LIB.wtp_crc32_batch_fixed(base + (i % 2) * N * P, P, P, N, op, sp)
    else:  # one 2 M launch
        W.LIB.wtp_crc32_batch_fixed(base, P, P, 2 * N, op, sp)


ref = {}
for kind, (_, base) in bufs.items():
    for _ in range(30):
        run(base, "two_m", 0)
    torch.cuda.synchronize()
    ref[kind] = out.clone()
kinds = list(bufs)
assert all(torch.equal(ref[k], ref[kinds[0]]) for k in kinds)
res = {f"{k}/{m}": [] for k in bufs for m in ("same", "alt", "two_m")}
for r in range(15):
    for m in ("same", "alt", "two_m"):
        for kind, (_, base) in bufs.items():
            s, e = TimingEvent(), TimingEvent()
            s.record(st)
            for i in range(10):
                run(base, m, i)
            e.record(st)
            torch.cuda.synchronize()
            res[f"{kind}/{m}"].append(s.elapsed_time(e) / 10 * 1e3)
print(json.dumps({"median_us_per_launch": {k: round(float(np.median(v)), 1) for k, v in res.items()},
                  "min_us": {k: round(float(np.min(v)), 1) for k, v in res.items()}}, indent=1))
