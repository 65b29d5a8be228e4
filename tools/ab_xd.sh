#!/bin/bash
# A/B of expand+depthwise builds on the C2 layer shapes (skip branch fused on
# the stride-2 layers): the in-tree library and each abx/libjabd_<name>.so,
# alternating, two rounds.  Usage on the GPU box: bash tools/ab_xd.sh name...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abxd
mkdir -p $O
export XD_SKIP_BRANCH=1
for r in 1 2; do
  timeout -k 10 120 python3 tools/convbench.py --set xd --reps 20 > $O/head_$r.log 2>&1 || exit 1
  for n in "$@"; do
    JABD_LIB=abx/libjabd_$n.so timeout -k 10 120 python3 tools/convbench.py --set xd --reps 20 > $O/${n}_$r.log 2>&1 || exit 1
  done
done
python3 - "$@" <<'PY'
import re, sys, glob
names = ["head"] + sys.argv[1:]
tab = {}
for n in names:
    for f in sorted(glob.glob(f"gpurun_out/abxd/{n}_*.log")):
        for l in open(f):
            m = re.match(r"(\S+\.xd)\s.*?\s([\d.]+) us", l)
            if m:
                tab.setdefault(m.group(1), {}).setdefault(n, []).append(float(m.group(2)))
print("%-8s" % "layer" + "".join("%18s" % n for n in names))
tot = {n: 0.0 for n in names}
for k, v in tab.items():
    print("%-8s" % k + "".join("%18s" % ("/".join("%.1f" % x for x in v.get(n, []))) for n in names))
    for n in names:
        tot[n] += min(v.get(n, [0]))
print("%-8s" % "sum(min)" + "".join("%18.1f" % tot[n] for n in names))
PY
