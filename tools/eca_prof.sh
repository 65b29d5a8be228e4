#!/bin/bash
# C4 kernel stats with the in-tree and the abx/libjabd_old.so builds (ECA reduction kernels)
set -o pipefail
mkdir -p gpurun_out/ecaab
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/eca_new -o run -- python3 tools/train_steps.py --kind mnv3 --steps 3 > gpurun_out/ecaab/prof_new.log 2>&1 &&
python3 tools/prof_summary.py /tmp/eca_new --csv gpurun_out/ecaab/new.csv > /dev/null 2>&1 &&
JABD_LIB=abx/libjabd_old.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/eca_old -o run -- python3 tools/train_steps.py --kind mnv3 --steps 3 > gpurun_out/ecaab/prof_old.log 2>&1 &&
python3 tools/prof_summary.py /tmp/eca_old --csv gpurun_out/ecaab/old.csv > /dev/null 2>&1
