#!/usr/bin/env python3
"""k_stream (forced) vs k_pieces on packed Zipf(1.1) batches of growing size: per-launch
time and read rate, to locate where the stream kernel falls off (diagnostic).
   python tools/stream_scale.py [--out f.json]"""
import argparse
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
import wtp_crc32 as W  # noqa: E402
from bench import TimingEvent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default=None)
ap.add_argument("--ns", default="1048576,2097152,4194304,8388608,15000000")
ap.add_argument("--modes", default="pieces,stream")
a = ap.parse_args()
assert W.LIB.wtp_init(0) == 0
st = torch.cuda.current_stream()
rows = []
for n in [int(x) for x in a.ns.split(",")]:
    lens = O.zipf_lengths(n, s=1.1)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=total)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    rb = total + 12 * n
    row = {"packets": n, "read_bytes": rb}
    row["payload_bytes"] = total
    for mode in a.modes.split(","):
        if mode == "stream":
            os.environ["WTP_STREAM_KERNEL"] = "1"
        f = lambda: W.crc32_batch_packed(d, total, do, dl, n, out)  # noqa: E731
        for _ in range(3):
            f()
        s, e = TimingEvent(), TimingEvent()
        s.record(st)
        for _ in range(10):
            f()
        e.record(st)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        os.environ.pop("WTP_STREAM_KERNEL", None)
        row[mode] = {"ms": round(ms, 4), "frac_hbm": round(rb / (ms * 1e-3) / 8e12, 4)}
    rows.append(row)
    print(json.dumps(row), flush=True)
    del d, do, dl, out
    torch.cuda.empty_cache()
if a.out:
    json.dump(rows, open(a.out, "w"), indent=1)
