#!/bin/bash
# fused previous project (blocks 1 -> 2): parity, then the C2 per-op table and bench both ways
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pre
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for r in 1 2; do
  JABD_FUSE_PRE=0 timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_off_$r.txt 2>&1 || exit 1
  timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_on_$r.txt 2>&1 || exit 1
  JABD_FUSE_PRE=0 timeout -k 10 200 python3 -u bench.py --no-train --no-nms --no-predict --no-cpu-baseline --r50-batch 0 > $O/bench_off_$r.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py --no-train --no-nms --no-predict --no-cpu-baseline --r50-batch 0 > $O/bench_on_$r.log 2>&1 || exit 1
done
echo rc=$?
