#!/bin/bash
# full GPU suite, then a stem rows A/B (abx/libjabd_r4.so: 4 output rows per thread)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 &&
JABD_LIB=abx/libjabd_r4.so timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/final/r4.log 2>&1 &&
timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/final/r2.log 2>&1 &&
JABD_LIB=abx/libjabd_r4.so timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/final/r4b.log 2>&1 &&
timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/final/r2b.log 2>&1
