"""Kernel time summary from a rocprofv3 --kernel-trace run (rocpd sqlite DB or
kernel_stats.csv): name, calls, total ms, average us, share.

  python3 tools/prof_summary.py <dir-with-run_results.db> [--top 40] [--csv out.csv]
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def load(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    agg = collections.defaultdict(lambda: [0, 0.0])
    if dbs:
        db = sqlite3.connect(dbs[0])
        cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
        name = "kernel_name" if "kernel_name" in cols else "name"
        for n, s, e in db.execute(f"select {name}, start, end from kernels"):
            agg[n][0] += 1
            agg[n][1] += (e - s) * 1e-6
        return agg
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Name"]][0] += int(r["Calls"])
            agg[r["Name"]][1] += float(r["TotalDurationNs"]) * 1e-6
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv")
    a = ap.parse_args()
    agg = load(a.dir)
    tot = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print("total kernel time %.2f ms over %d kernels" % (tot, sum(v[0] for v in agg.values())))
    for n, (c, t) in rows[:a.top]:
        print("%8.2f ms %5.1f%% %6d calls %9.1f us avg  %s" % (t, 100 * t / tot, c, 1e3 * t / c, n[:110]))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, (c, t) in rows:
                w.writerow([n, c, int(t * 1e6), t * 1e6 / c, 100 * t / tot])


if __name__ == "__main__":
    main()
