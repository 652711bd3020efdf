#!/usr/bin/env python3
"""Mean/median duration of one kernel over bench.py's timed window, from a rocprofv3
--kernel-trace CSV.  bench.py launches the kernel `skip` times while it settles
(warmup_run in its JSON line), then `steps` timed launches, then the read-ceiling
probe's interleaved launches; the --stats average covers all of them.
usage: rocprof_window.py <kernel_trace.csv> <kernel substring> <steps> <out.json> [skip]
(without skip: the last `steps` launches)"""
import csv
import json
import statistics
import sys

src, name, steps, dst = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
skip = int(sys.argv[5]) if len(sys.argv) > 5 else None
rows = sorted((r for r in csv.DictReader(open(src)) if name in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
win = us[skip:skip + steps] if skip is not None else us[-steps:]
lo = skip if skip is not None else len(us) - steps
out = {"kernel": name, "launches": len(us), "window": [lo, lo + len(win)],
       "window_mean_us": round(statistics.mean(win), 2), "window_median_us": round(statistics.median(win), 2),
       "all_mean_us": round(statistics.mean(us), 2),
       "before_window_mean_us": round(statistics.mean(us[:lo]), 2) if lo > 0 else None,
       "source": src}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out))
