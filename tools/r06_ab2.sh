#!/bin/bash
# Round-6 A/B 2: in-tree = expdw1 8-channel tail stage for Cin 24 (KCC 2 forms).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for r in 1 2; do
  JABD_LIB=abx/libjabd_base.so timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_base_$r.txt 2>&1 || exit 1
  timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_new_$r.txt 2>&1 || exit 1
  JABD_LIB=abx/libjabd_base.so timeout -k 10 120 python3 tools/convbench.py --set xd --reps 20 > $O/xd_base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/convbench.py --set xd --reps 20 > $O/xd_new_$r.log 2>&1 || exit 1
done
echo rc=$?
