#!/usr/bin/env python3
"""HBM read bytes per kernel from tools/gpu_c5_tcc.sh's passes: median per dispatch of
TCC_EA0_RDREQ (n), TCC_EA0_RDREQ_32B (n32), TCC_BUBBLE (n128) and FETCH_SIZE, and
   bytes = 32 n32 + 64 (n - n32 - n128) + 128 n128
beside the guide's streaming correction 2 * FETCH_SIZE * 1024.
  python tools/tcc_bytes.py gpurun_out/tcc"""
import csv
import glob
import json
import statistics
import sys

d = sys.argv[1]
per = {}  # (kernel, counter) -> {dispatch: value}
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        kern = "verify" if "VerifyBEpi" in k else ("c5" if "k_pieces" in k and "ArrayProvL" in k else None)
        if kern is None:
            continue
        per.setdefault((kern, r["Counter_Name"]), {}).setdefault(r["Dispatch_Id"], 0.0)
        per[(kern, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
algo = {"verify": 1048576 * 1472 + 4 * 1048576, "c5": 142102337 + 12 * 1048576}
out = {}
for kern in ("verify", "c5"):
    m = {c: statistics.median(v.values()) for (k, c), v in per.items() if k == kern}
    row = {"counters_median_per_dispatch": m, "algorithmic_read_bytes": algo[kern]}
    if {"TCC_EA0_RDREQ", "TCC_EA0_RDREQ_32B", "TCC_BUBBLE"} <= m.keys():
        n, n32, n128 = m["TCC_EA0_RDREQ"], m["TCC_EA0_RDREQ_32B"], m["TCC_BUBBLE"]
        b = 32 * n32 + 64 * (n - n32 - n128) + 128 * n128
        row["bytes_by_request_size"] = int(b)
        row["ratio_by_request_size"] = round(b / algo[kern], 4)
    if "FETCH_SIZE" in m:
        row["bytes_2x_fetch_size"] = int(2 * m["FETCH_SIZE"] * 1024)
        row["ratio_2x_fetch_size"] = round(2 * m["FETCH_SIZE"] * 1024 / algo[kern], 4)
    out[kern] = row
print(json.dumps(out, indent=1))
