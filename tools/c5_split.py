#!/usr/bin/env python3
"""Where the C5 time goes: the mixed-length kernel timed on length classes of the same
Zipf batch (same device buffer, compacted offset/length arrays per class).

  python tools/c5_split.py [--s 1.1] [--out f.json]    (WTP_LIB selects an A/B build)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402
from bench_configs import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--s", type=float, default=1.1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert W.LIB.wtp_init(0) == 0
    n = 1 << 20
    lens = O.zipf_lengths(n, s=a.s)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=total)
    host = d[:total].cpu().numpy()
    res = []
    classes = [("all", 0, 1 << 20), ("<16", 0, 16), ("<64", 0, 64), ("<256", 0, 256), (">=64", 64, 1 << 20),
               (">=256", 256, 1 << 20), (">=1024", 1024, 1 << 20), ("==1456", 1456, 1457)]
    for name, lo, hi in classes:
        sel = np.nonzero((lens >= lo) & (lens < hi))[0]
        m = int(sel.size)
        if m == 0:
            continue
        so, sl = offs[sel].copy(), lens[sel].copy()
        do = torch.from_numpy(so.view(np.int64)).cuda()
        dl = torch.from_numpy(sl.view(np.int32)).cuda()
        out = torch.empty(m, dtype=torch.int32, device="cuda")
        f = lambda: W.crc32_batch_var(d, total, do, dl, m, out)  # noqa: E731
        med, mean = timed(f, 100)
        got = out.cpu().numpy().view(np.uint32)
        idx = np.random.default_rng(3).integers(0, m, 500)
        ok = bool(np.array_equal(got[idx], O.batch_var(host, so[idx], sl[idx])))
        by = int(sl.sum())
        r = {"class": name, "packets": m, "bytes": by, "ms": round(mean, 4),
             "read_GBps": round((by + 12 * m) / (mean * 1e-3) / 1e9, 1),
             "ns_per_packet": round(mean * 1e6 / m, 4), "parity": ok}
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"lib": os.environ.get("WTP_LIB", "product"), "s": a.s, "results": res}, fh, indent=1)


if __name__ == "__main__":
    main()
