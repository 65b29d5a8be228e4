#!/bin/bash
# Round-6 A/B 1: in-tree = expdw1 8-channel tail + channel-range split + stem 8-byte loads.
# Parity tests on the in-tree build, the xd layer A/B (base / tail8 / split / in-tree),
# and the C2 per-op table for base vs in-tree (two rounds each).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for r in 1 2; do
  JABD_LIB=abx/libjabd_base.so timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_base_$r.txt 2>&1 || exit 1
  timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_new_$r.txt 2>&1 || exit 1
done &&
cp abx/libjabd_base.so /tmp/libjabd_head.so &&
for r in 1 2; do
  for n in base tail8 split stem; do
    JABD_LIB=abx/libjabd_$n.so timeout -k 10 120 python3 tools/convbench.py --set xd --reps 20 > $O/xd_${n}_$r.log 2>&1 || exit 1
  done
done
echo rc=$?
