#!/bin/bash
# bn3 backward link (dz + sums from the next bottleneck's conv1 data gradient): parity, C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bn3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train.py -m gpu -k "r50" > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_size.py tests/test_train_ops.py -m gpu > $O/tests2.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_on_$i.log 2>&1 &&
JABD_R50_BN3_LINK=0 timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_off_$i.log 2>&1 || exit 1
done
echo rc=$?
