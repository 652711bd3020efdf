#!/usr/bin/env python3
"""Per-wave phase times of the general kernel on C5-shaped batches (tools/pprobe.hip):
entry -> wave split -> LDS fill -> first round -> last round, from 100 MHz stamps.
  python tools/pprobe.py [--s 1.1] [--n 1048576] [--uniform L]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--s", type=float, default=1.1)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--uniform", type=int, default=0)
a = ap.parse_args()
L = C.CDLL(os.path.join(ROOT, "tools", "bin", "libpprobe.so"))
assert L.wtp_init(0) == 0
lens = np.full(a.n, a.uniform, np.uint32) if a.uniform else O.zipf_lengths(a.n, s=a.s).astype(np.uint32)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
L.wtp_synth_fill(C.c_void_p(d.data_ptr()), C.c_uint64(0), C.c_uint64(total), C.c_uint64(0x5EED), None)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(a.n, dtype=torch.int32, device="cuda")
st = torch.zeros(256 * 16 * 8, dtype=torch.int64, device="cuda")
assert L.pprobe_set(C.c_void_p(st.data_ptr())) == 0
call = lambda: L.wtp_crc32_batch_var(C.c_void_p(d.data_ptr()), C.c_size_t(total), C.c_void_p(do.data_ptr()),  # noqa
                                     C.c_void_p(dl.data_ptr()), C.c_size_t(a.n), C.c_void_p(out.data_ptr()), None)
for _ in range(20):
    assert call() == 0
torch.cuda.synchronize()
s = st.cpu().numpy().reshape(256, 16, 8).astype(np.int64)
live = s[:, :, 0] > 0
t0 = s[:, :, 0][live].min()
ph = {k: (s[:, :, k][live] - t0) / 100.0 for k in range(6)}  # microseconds
print(f"n={a.n} bytes={total} waves={live.sum()}")
for k, name in enumerate(["entry", "split", "fill", "loop0", "round1", "end"]):
    v = ph[k]
    print(f"  {name:7s} min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f} us")
r = s[:, :, 6][live]
dur = (s[:, :, 5][live] - s[:, :, 3][live]) / 100.0
print(f"  rounds/wave min {r.min()} mean {r.mean():.1f} max {r.max()}; loop us mean {dur.mean():.2f} max {dur.max():.2f};"
      f" us/round mean {np.mean(dur / np.maximum(r, 1)):.2f}")
print(f"  packets/wave min {s[:, :, 7][live].min()} max {s[:, :, 7][live].max()}")
# workgroup ends (last wave of each workgroup): the launch waits for the slowest
ends = np.where(live, (s[:, :, 5] - t0) / 100.0, -1.0).max(axis=1)
ends = ends[ends >= 0]
print(f"  workgroup end min {ends.min():.2f} mean {ends.mean():.2f} p90 {np.percentile(ends, 90):.2f} "
      f"max {ends.max():.2f} us (perfect cross-workgroup balance would end near the mean)")
if os.environ.get("PPROBE_DUMP"):
    np.save(os.environ["PPROBE_DUMP"], s)
