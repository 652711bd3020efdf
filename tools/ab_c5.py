#!/usr/bin/env python3
"""Interleaved A/B of the mixed-length path (config C5) across the libraries in
a3-reliable-transport_amd/lib/ab/*.so, in one process on one box: each library is loaded
with ctypes (RTLD_LOCAL: separate device state), the same Zipf batch is timed
alternately (A B C ... A B C ...), and every library's output must equal the first's.
  python tools/ab_c5.py [--s 1.1] [--reps 5] [--entry var|packed]
(--entry packed reaches the stream kernel only with WTP_STREAM_KERNEL=1 in the
environment; below 2 GiB wtp_crc32_batch_packed otherwise takes the piece kernel)"""
import argparse
import ctypes as C
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--s", type=float, default=1.1)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--entry", default="var", choices=["var", "packed"])
a = ap.parse_args()
libs = sorted(glob.glob(os.path.join(ROOT, "a3-reliable-transport_amd", "lib", "ab", "*.so")))
L = {os.path.basename(p)[:-3]: C.CDLL(p) for p in libs}
for lib in L.values():
    assert lib.wtp_init(0) == 0
lens = O.zipf_lengths(a.n, s=a.s).astype(np.uint32)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
first = next(iter(L.values()))
first.wtp_synth_fill(C.c_void_p(d.data_ptr()), C.c_uint64(0), C.c_uint64(total), C.c_uint64(0x5EED), None)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
outs = {k: torch.zeros(a.n, dtype=torch.int32, device="cuda") for k in L}
torch.cuda.synchronize()


def call(k):
    f = L[k].wtp_crc32_batch_packed if a.entry == "packed" else L[k].wtp_crc32_batch_var
    return f(C.c_void_p(d.data_ptr()), C.c_size_t(total), C.c_void_p(do.data_ptr()),
                                    C.c_void_p(dl.data_ptr()), C.c_size_t(a.n), C.c_void_p(outs[k].data_ptr()), None)


res = {k: [] for k in L}
NS = 100
for rep in range(a.reps):
    for k in L:
        for _ in range(5):
            assert call(k) == 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(NS + 1)]
        ev[0].record()
        for i in range(NS):
            call(k)
            ev[i + 1].record()
        torch.cuda.synchronize()
        t = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(NS))
        res[k].append(t[NS // 2])
ref = outs[next(iter(L))].cpu()
for k in L:
    same = bool(torch.equal(outs[k].cpu(), ref))
    m = np.mean(res[k])
    print(f"{k:14s} median-of-medians {np.median(res[k]) * 1e3:7.2f} us  mean {m * 1e3:7.2f} us  "
          f"reps {[round(x * 1e3, 1) for x in res[k]]}  same-as-first {same}", flush=True)
