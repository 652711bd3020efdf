#!/usr/bin/env python3
"""Split rocprofv3 --pmc counter CSVs of tools/tl_probe.py by phase (its fixed dispatch
order per kernel) and report the median per launch of every counter, per 1 M packets.

    tl_summary.py <phases.json> <out.json> <counter_collection.csv>...
"""
import csv
import json
import statistics
import sys

phases = json.load(open(sys.argv[1]))["order"]
dst = sys.argv[2]
per = {}  # (kernel kind, dispatch id) -> {counter: value}
for src in sys.argv[3:]:
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name", "")
        kind = "crc" if "k_fixed_braid" in name else ("probe" if "read_xor" in name else None)
        if kind is None:
            continue
        d = per.setdefault((src, kind, int(r["Dispatch_Id"])), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])

out = {}
for src in sys.argv[3:]:
    for kind in ("crc", "probe"):
        ds = sorted(k[2] for k in per if k[0] == src and k[1] == kind)
        i = 0
        for ph in (p for p in phases if p["kernel"] == kind):
            chunk = ds[i:i + ph["launches"]]
            i += ph["launches"]
            if ph["phase"].endswith("warm"):
                continue
            scale = (1 << 20) / ph["packets_per_launch"]
            row = out.setdefault(ph["phase"], {"time_us_per_1M": ph["median_us_per_1M"]})
            names = set().union(*(per[(src, kind, d)] for d in chunk)) if chunk else set()
            for c in sorted(names):
                v = [per[(src, kind, d)].get(c, 0.0) for d in chunk]
                row[c + "_per_1M"] = round(statistics.median(v) * scale, 1)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
