#!/bin/bash
# sum_multi with 16-byte lanes: bit-exactness test and the C3 step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sum4
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_ops.py tests/test_train.py -m gpu > $O/tests.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_$i.log 2>&1 || exit 1
done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/sum4prof -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/prof.log 2>&1 &&
python3 tools/prof_summary.py /tmp/sum4prof > $O/summary.txt
echo rc=$?
