#!/bin/bash
# expdw1 8-channel tail stage: parity (abx/libjabd_tail8.so) + per-layer A/B vs the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tail8
mkdir -p $O
JABD_LIB=abx/libjabd_split.so timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 bash tools/ab_xd.sh tail8 split > $O/ab.txt 2>&1
echo rc=$?
