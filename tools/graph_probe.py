#!/usr/bin/env python3
"""Can bench.py's timed steps run as one HIP graph (K kernel launches, each bracketed by
timing-only events), and what does it save per step?  Interleaved: K stream launches with
per-launch events (bench.py's current timed region) vs one replay of a captured graph of
the same K launches and events; wall time per step and the events' kernel times.
    graph_probe.py [--k 20] [--reps 10]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
P, n = 1456, 1 << 20
buf = torch.empty(n * P + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(buf, nbytes=n * P)
out = torch.empty(n, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
for _ in range(200):
    W.crc32_batch_fixed(buf, P, P, n, out, s)
torch.cuda.synchronize()
want = out.clone()

ev_s = [TimingEvent() for _ in range(a.k)]
ev_e = [TimingEvent() for _ in range(a.k)]


def steps():
    for i in range(a.k):
        ev_s[i].record(s)
        W.crc32_batch_fixed(buf, P, P, n, out, s)
        ev_e[i].record(s)


res = {"stream": {"wall_us": [], "kern_us": []}}
g = None
try:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        steps()
    res["graph"] = {"wall_us": [], "kern_us": []}
except Exception as e:  # noqa: BLE001
    res["graph_error"] = f"{e.__class__.__name__}: {e}"[:300]
    g = None
torch.cuda.synchronize()
for _ in range(a.reps):
    for mode in (("stream", "graph") if g is not None else ("stream",)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "stream":
            steps()
        else:
            g.replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res[mode]["wall_us"].append(el / a.k * 1e6)
        try:
            res[mode]["kern_us"].append(float(np.mean([x.elapsed_time(y) for x, y in zip(ev_s, ev_e)])) * 1e3)
        except RuntimeError as e:
            res[mode]["events_error"] = str(e)[:200]
assert torch.equal(out, want)
summ = {}
for m, v in res.items():
    if isinstance(v, dict):
        summ[m] = {k: round(float(np.median(x)), 2) for k, x in v.items() if isinstance(x, list) and x}
        summ[m].update({k: x for k, x in v.items() if not isinstance(x, list)})
    else:
        summ[m] = v
print(json.dumps(summ, indent=1))
