#!/usr/bin/env python3
"""Per-kernel duration summary (count, mean, median, p10, p90 in us) from a rocprofv3
rocpd database (the default output format of this image's rocprofv3).
  python tools/kstats.py <dir-or-db> [--grid]   (--grid splits by grid size)"""
import glob
import os
import sqlite3
import sys

import numpy as np

p = sys.argv[1]
dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
by = {}
for db in dbs:
    c = sqlite3.connect(db)
    for name, dur, gx, wx in c.execute("select name, duration, grid_x, workgroup_x from kernels"):
        key = name[:90] + (f" grid {gx // max(wx, 1)}x{wx}" if "--grid" in sys.argv else "")
        by.setdefault(key, []).append(dur / 1e3)
print(f"{'count':>6} {'mean':>9} {'median':>9} {'p10':>9} {'p90':>9}  kernel (us)")
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    a = np.array(v)
    print(f"{a.size:6d} {a.mean():9.2f} {np.median(a):9.2f} {np.percentile(a, 10):9.2f} {np.percentile(a, 90):9.2f}  {k}")
