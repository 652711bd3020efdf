#!/usr/bin/env python3
"""Where does the C4 per-rank step lose against a plain 2 M launch?  One process, one
2 M x 1456 B buffer, interleaved rounds of 10 steps: (a) plain launches on torch's
stream, all CUs' rule (reserve 0); (b) the same with 8 CUs reserved; (c) on a side
stream with 8 reserved; (d) bench.py's Pipe step with the one-rank RCCL gather every 2
steps.  Event pair around each 10-step run only.  Diagnostic."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import shard  # noqa: E402
import wtp_crc32 as W  # noqa: E402

P, N = 1456, 2 * 1048576
torch.cuda.set_device(0)
bench.init_one_rank_group(0)
assert W.LIB.wtp_init(0) == 0
dev = torch.device("cuda", 0)
buf = torch.empty(N * P + 64, dtype=torch.uint8, device=dev)
W.synth_fill(buf, nbytes=N * P)
out = torch.empty(N, dtype=torch.int32, device=dev)
main_st = torch.cuda.current_stream()
side = torch.cuda.Stream()
gathered = torch.empty(2 * 2 * N, dtype=torch.int32, device=dev)
pipe = bench.Pipe(W, shard, [buf], N, side, True, 1, 0, gathered, dev, every=2)


def run(mode, k=10):
    if mode == "plain":
        W.reserve_cus(0, 0)
        for _ in range(k):
            W.crc32_batch_fixed(buf, P, P, N, out, main_st)
        return main_st
    if mode == "reserve8":
        W.reserve_cus(8, 0)
        for _ in range(k):
            W.crc32_batch_fixed(buf, P, P, N, out, main_st)
        return main_st
    if mode == "side_reserve8":
        W.reserve_cus(8, 0)
        for _ in range(k):
            W.crc32_batch_fixed(buf, P, P, N, out, side)
        return side
    W.reserve_cus(8, 0)  # pipe with gather
    for _ in range(k):
        pipe.step()
    return side


modes = ["plain", "reserve8", "side_reserve8", "pipe_gather"]
for m in modes:
    run(m, 20)
pipe.drain()
torch.cuda.synchronize()
res = {m: [] for m in modes}
for r in range(12):
    for m in modes:
        st = side if m in ("side_reserve8", "pipe_gather") else main_st
        a, b = bench.TimingEvent(), bench.TimingEvent()
        torch.cuda.synchronize()
        a.record(st)
        run(m)
        b.record(st)
        if m == "pipe_gather":
            pipe.drain()
        torch.cuda.synchronize()
        res[m].append(a.elapsed_time(b) / 10)
W.reserve_cus(0, 0)
print(json.dumps({"ms_per_step_median": {m: round(float(np.median(v)), 5) for m, v in res.items()},
                  "ms_per_step_min": {m: round(float(np.min(v)), 5) for m, v in res.items()}}, indent=1))
import torch.distributed as dist  # noqa: E402
dist.destroy_process_group()
