#!/bin/bash
# ECA backward reduction A/B: ECA / training parity tests, then C4 step time and
# the two kernels' durations (in-tree vs abx/libjabd_old.so)
set -o pipefail
mkdir -p gpurun_out/ecaab
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_train_ops.py tests/test_train.py tests/test_modules.py -x -q -m gpu -k "eca or train or block" --timeout 120 --timeout-method thread > gpurun_out/ecaab/t.log 2>&1 &&
for i in 1 2; do
  JABD_LIB=abx/libjabd_old.so timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 >> gpurun_out/ecaab/c4_old.log 2>&1 &&
  timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 >> gpurun_out/ecaab/c4_new.log 2>&1 || exit 1
done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/eca_prof -o run -- python3 tools/train_steps.py --kind mnv3 --steps 3 > gpurun_out/ecaab/prof.log 2>&1 &&
python3 tools/prof_summary.py /tmp/eca_prof > gpurun_out/ecaab/summary.txt 2>&1
