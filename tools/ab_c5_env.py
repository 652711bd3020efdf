#!/usr/bin/env python3
"""C5 (mixed lengths, wtp_crc32_batch_var) through the two mixed-length kernels of ONE
library, interleaved in one process: k_pieces (default) and k_braid_var
(WTP_BRAID_VAR=1, read by the library at every call).  Each kernel's whole output is
checked against the CPU oracle; timings are medians of back-to-back calls and of HIP
graph replays.
  python tools/ab_c5_env.py [--s 1.1 1.0] [--reps 5] [--n 1048576]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--s", type=float, nargs="+", default=[1.1, 1.0])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--out", default=None)
a = ap.parse_args()
KERNELS = {"braid_var": "1", "pieces": "0"}
res = {}
for s in a.s:
    lens = O.zipf_lengths(a.n, s=s).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    host = O.synth_fill_np(total)
    want = O.batch_var(host, offs, lens)
    d = torch.from_numpy(host).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(a.n, dtype=torch.int32, device="cuda")

    def call():
        W.crc32_batch_var(d, total, do, dl, a.n, out)

    row = {}
    for name, env in KERNELS.items():
        os.environ["WTP_BRAID_VAR"] = env
        out.zero_()
        call()
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        row[name] = {"exact": bool(bad.size == 0), "mismatches": int(bad.size), "first_bad": bad[:8].tolist(),
                     "b2b_us": [], "graph_us": []}
    for rep in range(a.reps):
        for name, env in KERNELS.items():
            os.environ["WTP_BRAID_VAR"] = env
            for _ in range(5):
                call()
            NS = 50
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(NS + 1)]
            ev[0].record()
            for i in range(NS):
                call()
                ev[i + 1].record()
            torch.cuda.synchronize()
            t = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(NS))
            row[name]["b2b_us"].append(round(t[NS // 2] * 1e3, 2))
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                call()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(20):
                        call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g.replay()
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            row[name]["graph_us"].append(round(e0.elapsed_time(e1) / 100 * 1e3, 2))
    for name in KERNELS:
        row[name]["b2b_median_us"] = float(np.median(row[name]["b2b_us"]))
        row[name]["graph_median_us"] = float(np.median(row[name]["graph_us"]))
    res[f"zipf{s}"] = {"n": a.n, "payload_bytes": total, "read_bytes": total + 12 * a.n, **row}
    print(json.dumps({f"zipf{s}": res[f"zipf{s}"]}), flush=True)
os.environ.pop("WTP_BRAID_VAR", None)
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
