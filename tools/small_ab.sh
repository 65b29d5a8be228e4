#!/bin/bash
# small-reduction A/B: BN / wgrad parity tests, then C4 kernel stats (in-tree vs abx/libjabd_old.so)
set -o pipefail
mkdir -p gpurun_out/smallab
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_train_ops.py tests/test_train_size.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/smallab/t.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/sm_new -o run -- python3 tools/train_steps.py --kind mnv3 --steps 3 > gpurun_out/smallab/prof_new.log 2>&1 &&
python3 tools/prof_summary.py /tmp/sm_new --csv gpurun_out/smallab/new.csv > /dev/null 2>&1 &&
JABD_LIB=abx/libjabd_old.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/sm_old -o run -- python3 tools/train_steps.py --kind mnv3 --steps 3 > gpurun_out/smallab/prof_old.log 2>&1 &&
python3 tools/prof_summary.py /tmp/sm_old --csv gpurun_out/smallab/old.csv > /dev/null 2>&1
