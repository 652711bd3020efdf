#!/usr/bin/env python3
"""Summarise tools/prof_sq.sh output: per kernel, the mean of each counter over its
dispatches (all passes merged).   usage: tools/sq_summary.py gpurun_out/<tag>/<path>"""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"][:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", d)
    for k, cs in acc.items():
        # values are per (dispatch, dimension): sum per dispatch = total / dispatches
        print(" ", k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {sum(v) / max(1, len(v) // max(1, 1)):.4g}  (n={len(v)})")
