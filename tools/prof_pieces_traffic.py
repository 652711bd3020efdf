#!/usr/bin/env python3
"""Driver for the general kernel's HBM-traffic attribution (rocprofv3 --pmc FETCH_SIZE):
three batches through k_pieces, a few launches each, in this order
  1. C5: 1 M packed Zipf(1.1) payloads (offset/length arrays)
  2. fixed: 1 M x 1456 B at a 1457-B stride (FixedProvL: no metadata loads)
  3. c5meta0: C5's lengths, but every offset 0 (every payload reads the same bytes: the
     launch's payload traffic is nil, what remains is metadata and its re-reads)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = 1 << 20
lens = O.zipf_lengths(n, s=1.1)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(d, nbytes=total)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(reps):
    W.crc32_batch_var(d, total, do, dl, n, out)
torch.cuda.synchronize()
f = torch.empty(n * 1457 + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(f, nbytes=n * 1457)
for _ in range(reps):
    W.crc32_batch_fixed(f, 1457, 1456, n, out)
torch.cuda.synchronize()
del f
z = torch.zeros(n, dtype=torch.int64, device="cuda")
for _ in range(reps):
    W.crc32_batch_var(d, total, z, dl, n, out)
torch.cuda.synchronize()
print("done")
