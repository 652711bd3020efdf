#!/usr/bin/env python3
"""Mean/median duration of one kernel over bench.py's timed window, from a rocprofv3
--kernel-trace CSV: the last `steps` launches (bench.py runs `warmup` launches first,
whose DVFS transient the --stats average includes).
usage: rocprof_window.py <kernel_trace.csv> <kernel substring> <steps> <out.json>"""
import csv
import json
import statistics
import sys

src, name, steps, dst = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
rows = sorted((r for r in csv.DictReader(open(src)) if name in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
win = us[-steps:]
out = {"kernel": name, "launches": len(us), "window": len(win),
       "window_mean_us": round(statistics.mean(win), 2), "window_median_us": round(statistics.median(win), 2),
       "all_mean_us": round(statistics.mean(us), 2), "warmup_mean_us": round(statistics.mean(us[:-steps]), 2) if len(us) > steps else None,
       "source": src}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out))
