#!/bin/bash
# stem A/B: parity tests + C2 per-op timing (new in-tree vs abx/libjabd_old.so)
set -o pipefail
mkdir -p gpurun_out/stem
timeout -k 10 300 python3 -u -m pytest tests/test_fused.py tests/test_modules.py tests/test_model.py -x -q -m gpu -k "stem or mnv3" --timeout 120 --timeout-method thread > gpurun_out/stem/t.log 2>&1 &&
JABD_LIB=abx/libjabd_old.so timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/stem/old.log 2>&1 &&
timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/stem/new.log 2>&1 &&
JABD_LIB=abx/libjabd_old.so timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/stem/old2.log 2>&1 &&
timeout -k 10 200 python3 -u tools/fwd_ops.py > gpurun_out/stem/new2.log 2>&1
