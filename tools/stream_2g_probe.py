#!/usr/bin/env python3
"""k_stream (forced) on packed Zipf(1.1) batches of n payloads, a few launches, for
counter passes around the 2 GiB buffer size (diagnostic):  stream_2g_probe.py n [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lens = O.zipf_lengths(n, s=1.1)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(d, nbytes=total)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(n, dtype=torch.int32, device="cuda")
os.environ["WTP_STREAM_KERNEL"] = "1"
for _ in range(reps):
    W.crc32_batch_packed(d, total, do, dl, n, out)
torch.cuda.synchronize()
print("done", n, total)
