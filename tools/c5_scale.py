#!/usr/bin/env python3
"""Cost model of the mixed-length kernel: packed batches through wtp_crc32_batch_var at
several sizes (fixed cost vs marginal cost) and with uniform lengths (per-packet vs
per-piece cost).   python tools/c5_scale.py [--out f.json]"""
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


def run(name, lens, d, res):
    n = int(lens.size)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    f = lambda: W.crc32_batch_var(d, total, do, dl, n, out)  # noqa: E731
    med, mean = timed(f, 100)
    got = out.cpu().numpy().view(np.uint32)
    idx = np.random.default_rng(3).integers(0, n, 300)
    host = d[: total].cpu().numpy()
    ok = bool(np.array_equal(got[idx], O.batch_var(host, offs[idx], lens[idx])))
    pieces = int(np.maximum(1, (lens.astype(np.int64) + 63) // 64).sum())
    r = {"case": name, "packets": n, "bytes": total, "pieces": pieces, "us": round(mean * 1e3, 2),
         "ns_per_piece": round(mean * 1e6 / pieces, 4), "read_GBps": round((total + 12 * n) / (mean * 1e-3) / 1e9, 1),
         "parity": ok}
    print(json.dumps(r), flush=True)
    res.append(r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert W.LIB.wtp_init(0) == 0
    big = 1 << 22
    zl = O.zipf_lengths(big, s=1.1)
    cap = int(zl.sum()) + 4096
    d = torch.empty(max(cap, (1 << 20) * 1456 + 64), dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=d.numel())
    res = []
    for k in (16, 18, 20, 21, 22):
        run(f"zipf1.1 n=2^{k}", zl[: 1 << k].copy(), d, res)
    for L in (1, 8, 32, 64, 65, 128, 256, 512, 1456):
        n = min(1 << 20, (1 << 27) // L)
        run(f"uniform L={L}", np.full(n, L, dtype=np.uint32), d, res)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
