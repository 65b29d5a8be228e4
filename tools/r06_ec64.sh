#!/bin/bash
# block 2's fused-project form with all 64 expanded channels in one 8-wave workgroup vs 32-channel chunks
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ec64
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for r in 1 2; do
  JABD_EXPDW_PRE_EC=32 timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_ec32_$r.txt 2>&1 || exit 1
  timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_ec64_$r.txt 2>&1 || exit 1
done
echo rc=$?
