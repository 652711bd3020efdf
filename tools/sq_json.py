#!/usr/bin/env python3
"""Per-dispatch counter means of the general-kernel profile (tools/prof_pieces.sh passes
+ a FETCH_SIZE pass over tools/prof_pieces.py) as JSON, one block per kernel, and the
derived figures DESIGN 7.9 uses (VALU busy share of SIMD time, VALU per payload byte, LDS
bank-conflict share, HBM read bytes with the gfx950 x2 FETCH_SIZE correction).
    sq_json.py <out.json> <label>=<dir> [<label>=<dir> ...]"""
import csv
import glob
import json
import sys
from collections import defaultdict

C5_PAYLOAD = 142_102_337  # bytes of payload in C5's 1 M Zipf(1.1) packets (tools/prof_pieces.py)
NAMES = {"k_fixed_braid": "k_fixed_braid<VerifyBEpi> (verify 1M)", "k_pieces": "k_pieces<ArrayProvL,CrcEpi> (C5 Zipf 1.1)"}

out = {"what": "per-dispatch counter means (rocprofv3 --pmc, one pass per line of tools/prof_pieces.sh, "
               "+ FETCH_SIZE), tools/sq_json.py"}
for arg in sys.argv[2:]:
    label, d = arg.split("=", 1)
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch, file) -> counter -> value
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((v for key, v in NAMES.items() if key in r["Kernel_Name"]), None)
            if k is None:
                continue
            per[(k, r["Dispatch_Id"], f)][r["Counter_Name"]] += float(r["Counter_Value"])
    blk = {}
    for (k, _d, _f), cs in per.items():
        for c, v in cs.items():
            blk.setdefault(k, defaultdict(list))[c].append(v)
    res = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in blk.items()}
    c5 = res.get(NAMES["k_pieces"])
    if c5 and "SQ_ACTIVE_INST_VALU" in c5 and "SQ_WAVE_CYCLES" in c5:
        w = c5.get("SQ_WAVES", 4096) / (256 * 4)  # waves per SIMD
        c5["derived"] = {
            "valu_active_share_of_simd_time": round(c5["SQ_ACTIVE_INST_VALU"] / c5["SQ_WAVE_CYCLES"] * w, 3),
            "valu_per_payload_byte": round(c5["SQ_INSTS_VALU"] / C5_PAYLOAD, 4),
            "lds_insts_per_payload_byte": round(c5.get("SQ_INSTS_LDS", 0) / C5_PAYLOAD, 4),
            "lds_bank_conflict_share": round(c5.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c5.get("SQ_LDS_IDX_ACTIVE", 1.0)), 3),
        }
        if "FETCH_SIZE" in c5:
            c5["derived"]["hbm_read_bytes_x2"] = int(2 * 1024 * c5["FETCH_SIZE"])
    out[label] = res
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps(out, indent=1)[:4000])
