"""Per-kernel average of rocprofv3 --pmc counters (counter_collection.csv).

  python3 tools/pmc_kernel.py <dir> [<dir> ...] --match expdw1 [--top 10]

Prints, per kernel name containing --match, the number of dispatches and the
mean value of every counter found under the given directories (one
directory per PMC pass).
"""
import argparse
import collections
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=10)
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "")
                if a.match in k:
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted(vals, key=lambda k: -len(next(iter(vals[k].values()))))[: a.top]
    for k in names:
        print(k[:110])
        for c, v in sorted(vals[k].items()):
            print(f"    {c:28s} n={len(v):4d} mean={sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
