#!/usr/bin/env python3
"""Do entry points that take stream-ordered scratch (hipMallocFromPoolAsync) replay
correctly from a captured HIP graph?  (1) wtp_crc32_batch_packed past 2 GiB (the device-
cut piece sub-launches' descriptors), (2) wtp_build_data_packets' slow path with no
length array (its CRC scratch).  Each: eager result, output cleared, one call captured
on a side stream (after an eager call on it), replayed, compared.  Diagnostic tool."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402


def replay_matches(call, out):
    call()
    torch.cuda.synchronize()
    want = out.clone()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        call()
    cs.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=cs):
            call()
    except Exception as e:  # noqa: BLE001
        return {"capture_error": f"{e.__class__.__name__}: {e}"[:300]}
    out.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    r = {"replay_equal": bool(torch.equal(out, want)), "nonzero_after_replay": int((out != 0).sum().item()),
         "elements": out.numel()}
    # stream order: a copy queued right behind the replay (no host sync in between) must
    # see the replay's results; events around the replay must bracket its work
    out.zero_()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    snap = out.clone()
    b.record()
    torch.cuda.synchronize()
    r["copy_behind_replay_equal"] = bool(torch.equal(snap, want))
    r["replay_plus_copy_ms"] = round(a.elapsed_time(b), 4)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    call()
    t1.record()
    torch.cuda.synchronize()
    r["eager_call_ms"] = round(t0.elapsed_time(t1), 4)
    return r


assert W.LIB.wtp_init(0) == 0
res = {}
n = 17_000_000
lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum())
d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(d, nbytes=total)
do = torch.from_numpy(offs.view(np.int64)).cuda()
dl = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.zeros(n, dtype=torch.int32, device="cuda")
res["packed_over_2gib"] = replay_matches(lambda: W.crc32_batch_packed(d, total, do, dl, n, out), out)
del d, do, dl, out
torch.cuda.empty_cache()
m = 50_001
pay = torch.empty(m * 1456 + 64, dtype=torch.uint8, device="cuda")
W.synth_fill(pay)
wire = torch.zeros(m * 1472 + 64, dtype=torch.uint8, device="cuda")
res["builder_slow_path_no_lengths"] = replay_matches(
    lambda: W.build_data_packets(pay[3:], m * 1456 - 100, 7, wire, 1472, None), wire)
print(json.dumps(res, indent=1))
