#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r50knobs
mkdir -p $O
timeout -k 10 200 python3 tools/convbench.py --set r50t --reps 10 > $O/base.log 2>&1 &&
JABD_M32_TM=2 timeout -k 10 200 python3 tools/convbench.py --set r50t --reps 10 > $O/tm2.log 2>&1 &&
JABD_CONV32=0 timeout -k 10 200 python3 tools/convbench.py --set r50t --reps 10 > $O/conv16.log 2>&1
echo rc=$?
