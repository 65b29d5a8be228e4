#!/bin/bash
# act-free GEMM epilogues (conv32 kEpiLin, conv_stream hoisted act): C2 per-op A/B vs HEAD, bit-identity, tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/epi
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_fused.py tests/test_model.py tests/test_modules.py tests/test_packing.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for r in 1 2; do
  JABD_LIB=abh/libjabd_head.so timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_head_$r.txt 2>&1 || exit 1
  timeout -k 10 150 python3 -u tools/fwd_ops.py > $O/fwd_new_$r.txt 2>&1 || exit 1
done &&
JABD_LIB=abh/libjabd_head.so timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/head > $O/head.log 2>&1 &&
timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/new > $O/new.log 2>&1 &&
python3 tools/m32s_ab.py --compare $O/head $O/new > $O/cmp.log 2>&1
echo rc=$?
