#!/usr/bin/env python3
"""Per-wave start/end times of the braided kernel (tools/pprobe.hip build) on the headline
batch, 1 M x 1456 B after `--warm` back-to-back launches (stamps of the last launch):
how long the slowest waves trail the rest.   python tools/bprobe.py [--n N] [--warm W]"""
import argparse
import ctypes as C
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--warm", type=int, default=100)
a = ap.parse_args()
L = C.CDLL(os.path.join(ROOT, "tools", "bin", os.environ.get("PPROBE_LIB", "libpprobe.so")))
assert L.wtp_init(0) == 0
d = torch.empty(a.n * 1456, dtype=torch.uint8, device="cuda")
L.wtp_synth_fill(C.c_void_p(d.data_ptr()), C.c_uint64(0), C.c_uint64(d.numel()), C.c_uint64(0x5EED), None)
out = torch.empty(a.n, dtype=torch.int32, device="cuda")
st = torch.zeros(256 * 16 * 8, dtype=torch.int64, device="cuda")
assert L.pprobe_set(C.c_void_p(st.data_ptr())) == 0
for _ in range(a.warm):
    assert L.wtp_crc32_batch_fixed(C.c_void_p(d.data_ptr()), C.c_size_t(1456), C.c_size_t(1456), C.c_size_t(a.n),
                                   C.c_void_p(out.data_ptr()), None) == 0
torch.cuda.synchronize()
s = st.cpu().numpy().reshape(256, 16, 8).astype(np.int64)[:, :8, :]  # 512-thread workgroups: 8 waves
t0 = s[:, :, 0][s[:, :, 0] > 0].min()
beg = (s[:, :, 3] - t0) / 100.0
end = (s[:, :, 5] - t0) / 100.0
print(f"n={a.n}: loop start max {beg.max():.2f} us; end min {end.min():.2f} med {np.median(end):.2f} "
      f"mean {end.mean():.2f} max {end.max():.2f} us")
ent = (s[:, :, 0] - t0) / 100.0
for k, nm in ((1, "after first loads issued"), (2, "after table fill (pre-barrier)")):
    v = (s[:, :, k] - t0) / 100.0
    print(f"  {nm}: min {v.min():.2f} med {np.median(v):.2f} max {v.max():.2f} us")
r1 = (s[:, :, 4] - t0) / 100.0
print(f"  entry min {ent.min():.2f} max {ent.max():.2f}; loop start min {beg.min():.2f} med {np.median(beg):.2f}; "
      f"first round done min {r1.min():.2f} med {np.median(r1):.2f} max {r1.max():.2f} us")
print("  end by wave//4:", [round(float(end[:, 4 * w:4 * w + 4].mean()), 2) for w in range(4)])
print("  end by wave%4:", [round(float(end[:, w::4].mean()), 2) for w in range(4)])
print("  end by xcd:", [round(float(end[x::8].mean()), 2) for x in range(8)])
if os.environ.get("PPROBE_DUMP"):
    np.save(os.environ["PPROBE_DUMP"], s)
