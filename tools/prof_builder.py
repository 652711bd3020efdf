#!/usr/bin/env python3
"""Driver for PMC passes over the fused DATA packet builder (1 M x 1456 B -> 1472-B wire
slots, 20 launches) and, for comparison, torch's device copy of the same payload bytes.
Run under rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE (one counter group per pass)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
import torch  # noqa: E402

import wtp_crc32 as W  # noqa: E402

n, stride = 1 << 20, 1472
assert W.LIB.wtp_init(0) == 0
wire = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
payload = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
W.synth_fill(payload)
wl = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
for _ in range(5):
    wire[:n * 1456].copy_(payload)
torch.cuda.synchronize()
print("ok")
