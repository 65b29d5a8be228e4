"""Per-dispatch durations of the kernels whose name contains a substring,
from a rocprofv3 --kernel-trace run directory (rocpd sqlite DB or the
kernel_trace.csv): name, grid, workgroup, duration; averaged per (name, grid).

  python3 tools/kernel_calls.py <run-dir> SUBSTRING [SUBSTRING ...]
"""
import collections
import csv
import glob
import os
import sqlite3
import sys

d, subs = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(list)
dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
if dbs:
    db = sqlite3.connect(dbs[0])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    gx = [c for c in cols if c.startswith("grid")]
    wx = [c for c in cols if c.startswith("workgroup")]
    q = f"select {name}, start, end, {', '.join(gx + wx) or '0'} from kernels"
    for r in db.execute(q):
        if any(s in r[0] for s in subs):
            agg[(r[0].split('(')[0][:70], tuple(r[3:]))].append((r[2] - r[1]) * 1e-3)
else:
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if any(s in n for s in subs):
                g = (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Workgroup_Size_X"))
                agg[(n.split('(')[0][:70], g)].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k, v in sorted(agg.items()):
    v = sorted(v)
    print(f"{k[0]:72s} {str(k[1]):40s} n={len(v):3d} med={v[len(v)//2]:9.1f} us min={v[0]:9.1f}")
