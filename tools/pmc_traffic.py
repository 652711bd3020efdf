#!/usr/bin/env python3
"""Per-launch HBM read traffic of the braided kernel from a rocprofv3 --pmc FETCH_SIZE
pass (gfx950 correction per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE is
in KiB and reports half the bytes of a wide coalesced streaming read, so bytes =
2 * FETCH_SIZE * 1024).  Writes profiles/pmc_traffic.json for bench.py, stamped with the
sha256 of the measured kernel's machine code in the library the pass ran (tools/codeobj.py):
bench.py reports the traffic only while the shipped kernel has the same code.

    pmc_traffic.py <counter_collection.csv> <out.json> <packets> [<lib.so>]"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import codeobj  # noqa: E402

src, dst, packets = sys.argv[1], sys.argv[2], int(sys.argv[3])
vals = {}
for r in csv.DictReader(open(src)):
    if "k_fixed_braid" not in r.get("Kernel_Name", ""):
        continue
    if r.get("Counter_Name") != "FETCH_SIZE":
        continue
    vals.setdefault(r["Dispatch_Id"], 0.0)
    vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
per = [v for v in vals.values()]
med = statistics.median(per)
out = {"packets": packets, "payload_bytes": packets * 1456, "dispatches": len(per),
       "FETCH_SIZE_KiB_median": med, "hbm_bytes_per_launch": int(2 * med * 1024),
       "correction": "bytes = 2 * FETCH_SIZE(KiB) * 1024 (gfx950 half-count of wide streaming reads)",
       "ratio_to_algorithmic": round(2 * med * 1024 / (packets * 1456), 4), "source": src}
lib = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "a3-reliable-transport_amd", "lib", "libwtp_crc32.so")
out["kernel_code"] = codeobj.kernel_code_sha256(lib, codeobj.HEADLINE_KERNEL)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out))
