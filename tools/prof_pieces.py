#!/usr/bin/env python3
"""Driver for counter profiles of the general kernel: receiver verify (1M x 1472-B
datagrams) and C5 (1M Zipf(1.1) packed payloads), a few launches each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, stride = 1 << 20, 1472
wire = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
payload = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
W.synth_fill(payload)
wl = torch.empty(n, dtype=torch.int32, device="cuda")
W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
ok = torch.empty(n, dtype=torch.uint8, device="cuda")
del payload
lens = O.zipf_lengths(n, s=1.1)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(d, nbytes=total)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(reps):
    W.verify_batch(wire, stride, wl, n, ok)
for _ in range(reps):
    W.crc32_batch_var(d, total, do, dl, n, out)
torch.cuda.synchronize()
print("verify ok:", int(ok.sum().item()) == n)
