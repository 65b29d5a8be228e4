#!/bin/bash
# per-layer GEMM efficiency at HEAD: R50 eval / C3 short-K forwards / C4 data gradients, weight gradients
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm
mkdir -p $O
timeout -k 10 200 python3 tools/convbench.py --set r50 --reps 10 > $O/r50.log 2>&1 &&
timeout -k 10 200 python3 tools/convbench.py --set r50t --reps 10 > $O/r50t.log 2>&1 &&
timeout -k 10 200 python3 tools/convbench.py --set tr --reps 10 > $O/tr.log 2>&1 &&
timeout -k 10 300 python3 tools/wgradbench.py > $O/wgrad.log 2>&1
echo rc=$?
