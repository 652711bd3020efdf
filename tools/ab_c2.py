#!/usr/bin/env python3
"""Interleaved A/B of the braided kernel on small batches (config C2: 64 K x 1456 B, and
other sizes) across a3-reliable-transport_amd/lib/ab/*.so in one process: per library,
launches replayed from a captured HIP graph (no host work between kernels), alternating
libraries per repetition; every library's CRCs must equal the first's.
  python tools/ab_c2.py [--n 65536] [--reps 5]"""
import argparse
import ctypes as C
import glob
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--G", type=int, default=50)
a = ap.parse_args()
libs = sorted(glob.glob(os.path.join(ROOT, "a3-reliable-transport_amd", "lib", "ab", "*.so")))
L = {os.path.basename(p)[:-3]: C.CDLL(p) for p in libs}
for lib in L.values():
    assert lib.wtp_init(0) == 0
d = torch.empty(a.n * 1456, dtype=torch.uint8, device="cuda")
first = next(iter(L.values()))
first.wtp_synth_fill(C.c_void_p(d.data_ptr()), C.c_uint64(0), C.c_uint64(d.numel()), C.c_uint64(0x5EED), None)
outs = {k: torch.zeros(a.n, dtype=torch.int32, device="cuda") for k in L}
torch.cuda.synchronize()
s = torch.cuda.Stream()
graphs = {}
for k, lib in L.items():
    def call(lib=lib, k=k):
        return lib.wtp_crc32_batch_fixed(C.c_void_p(d.data_ptr()), C.c_size_t(1456), C.c_size_t(1456), C.c_size_t(a.n),
                                         C.c_void_p(outs[k].data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    for _ in range(3):
        assert call() == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.G):
            call()
    graphs[k] = g
res = {k: [] for k in L}
for rep in range(a.reps):
    for k, g in graphs.items():
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / (10 * a.G) * 1e3)
ref = outs[next(iter(L))].cpu()
for k in L:
    print(f"{k:14s} n={a.n} graph us/launch median {np.median(res[k]):7.2f}  reps {[round(x, 2) for x in res[k]]}  "
          f"same-as-first {bool(torch.equal(outs[k].cpu(), ref))}", flush=True)
