#!/usr/bin/env python3
"""Where does k_stream slow down past a 2 GiB buffer?  15.9 M packed Zipf(1.1) payloads
(2.16 GB), the forced stream kernel on: the whole batch; its first half (offsets below
1.1 GB) with the whole buffer as the view; its second half with the whole buffer; the
second half through a rebased base pointer (a < 2 GiB view).  Diagnostic."""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 15_900_000
lens = O.zipf_lengths(n, s=1.1)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(d, nbytes=total)
out = torch.empty(n, dtype=torch.int32, device="cuda")
os.environ["WTP_STREAM_KERNEL"] = "1"
st = torch.cuda.current_stream()
h = n // 2
cases = {
    "all": (d, total, offs, lens, n, out),
    "first_half_full_view": (d, total, offs[:h], lens[:h], h, out),
    "second_half_full_view": (d, total, offs[h:], lens[h:], n - h, out[h:]),
    "second_half_rebased": (d[int(offs[h]):], total - int(offs[h]), offs[h:] - offs[h], lens[h:], n - h, out[h:]),
}
res = {"packets": n, "bytes": total}
for name, (b, bb, o, l, m, ot) in cases.items():
    do = torch.from_numpy(np.ascontiguousarray(o).view(np.int64)).cuda()
    dl = torch.from_numpy(np.ascontiguousarray(l).view(np.int32)).cuda()
    f = lambda: W.crc32_batch_packed(b, bb, do, dl, m, ot)  # noqa: E731
    f()
    torch.cuda.synchronize()
    s, e = TimingEvent(), TimingEvent()
    s.record(st)
    for _ in range(3):
        f()
    e.record(st)
    torch.cuda.synchronize()
    res[name] = round(s.elapsed_time(e) / 3, 4)
    print(name, res[name], flush=True)
print(json.dumps(res))
