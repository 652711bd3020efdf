#!/usr/bin/env python3
"""One config's kernel, launched `--reps` times back to back, for a rocprofv3 --pmc pass
(one config per process so each counter file holds one workload):

    rocprofv3 --pmc FETCH_SIZE -d <dir> -o <row> -- python3 tools/pmc_configs.py <row>
    rows: c2 | c5_1.1 | c5_1.0 | verify | build

Inputs are the configs leg's (tools/config_legs.py: device generator, Zipf lengths).  Then
`pmc_configs.py --summarize <out.json> <row>=<dir> ...` reads the counter CSVs and writes
per-launch HBM bytes and their ratio to each row's algorithmic bytes (gfx950 correction as
tools/pmc_traffic.py: bytes = 2 * FETCH_SIZE KiB * 1024 for wide streaming reads;
WRITE_SIZE likewise in KiB, uncorrected)."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 1456
N1M = 1 << 20


def algorithmic(row: str) -> dict:
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import config_legs as CL
    if row == "c2":
        return {"read": 65536 * P, "write": 65536 * 4}
    if row.startswith("c5_"):
        lens = CL.zipf_lengths(N1M, s=float(row[3:]))
        return {"read": int(lens.sum()) + 12 * N1M, "write": 4 * N1M}
    if row == "verify":
        return {"read": N1M * (16 + P + 4), "write": N1M}
    if row == "build":
        return {"read": N1M * P, "write": N1M * (16 + P + 4)}
    raise SystemExit(f"unknown row {row}")


def run(row: str, reps: int) -> None:
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import config_legs as CL
    import wtp_crc32 as W
    assert W.LIB.wtp_init(0) == 0
    if row == "c2":
        n = 65536
        buf = torch.empty(n * P, dtype=torch.uint8, device="cuda")
        W.synth_fill(buf)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        f = lambda: W.crc32_batch_fixed(buf, P, P, n, out)  # noqa: E731
    elif row.startswith("c5_"):
        lens = CL.zipf_lengths(N1M, s=float(row[3:]))
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
        total = int(lens.sum())
        d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        W.synth_fill(d, nbytes=total)
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        out = torch.empty(N1M, dtype=torch.int32, device="cuda")
        f = lambda: W.crc32_batch_packed(d, total, do, dl, N1M, out)  # noqa: E731
    else:
        payload = torch.empty(N1M * P, dtype=torch.uint8, device="cuda")
        W.synth_fill(payload)
        wire = torch.empty(N1M * (16 + P), dtype=torch.uint8, device="cuda")
        wl = torch.empty(N1M, dtype=torch.int32, device="cuda")
        W.build_data_packets(payload, N1M * P, 0, wire, 16 + P, wl)
        ok = torch.empty(N1M, dtype=torch.uint8, device="cuda")
        if row == "verify":
            f = lambda: W.verify_batch(wire, 16 + P, wl, N1M, ok)  # noqa: E731
        else:
            f = lambda: W.build_data_packets(payload, N1M * P, 0, wire, 16 + P, wl)  # noqa: E731
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    print(json.dumps({"row": row, "reps": reps, "kernel": W.LIB.wtp_last_kernel().decode()}))


def summarize(dst: str, pairs: list) -> None:
    out = {"what": "per-launch HBM traffic of each configs-leg kernel (rocprofv3 --pmc, one config per process)",
           "correction": "read bytes = 2 * FETCH_SIZE(KiB) * 1024 (gfx950, wide streaming reads); "
                         "write bytes = WRITE_SIZE(KiB) * 1024", "rows": {}}
    for pair in pairs:
        row, d = pair.split("=", 1)
        alg = algorithmic(row)
        r = {"algorithmic": alg}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = {}
            names = {}
            for x in csv.DictReader(open(f)):
                k = x.get("Kernel_Name", "")
                if not ("k_fixed_braid" in k or "k_pieces" in k or "k_stream" in k):
                    continue
                c = x.get("Counter_Name")
                per.setdefault(c, {}).setdefault(x["Dispatch_Id"], 0.0)
                per[c][x["Dispatch_Id"]] += float(x["Counter_Value"])
                names[k.split("(")[0]] = 1
            for c, v in per.items():
                med = statistics.median(v.values())
                if c == "FETCH_SIZE":
                    b = 2 * med * 1024
                    r["read_bytes_per_launch"] = int(b)
                    r["read_ratio"] = round(b / alg["read"], 4)
                elif c == "WRITE_SIZE":
                    b = med * 1024
                    r["write_bytes_per_launch"] = int(b)
                    r["write_ratio"] = round(b / alg["write"], 4)
                r[c + "_dispatches"] = len(v)
            if names:
                r["kernels"] = sorted(names)
        out["rows"][row] = r
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--summarize":
        summarize(sys.argv[2], sys.argv[3:])
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
