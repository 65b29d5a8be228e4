#!/bin/bash
# residual rows prefetched before the epilogue's LDS round trip: parity, bit-identity vs HEAD, C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/resp
mkdir -p $O
true || timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train.py tests/test_train_ops.py tests/test_model.py -m gpu > $O/tests.log 2>&1 &&
JABD_LIB=abh/libjabd_head.so timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/head > $O/head.log 2>&1 &&
timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/new > $O/new.log 2>&1 &&
{ python3 tools/m32s_ab.py --compare $O/head $O/new > $O/cmp.log 2>&1; true; } &&
for i in 1 2; do
timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_new_$i.log 2>&1 &&
JABD_LIB=abh/libjabd_head.so timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_head_$i.log 2>&1 || exit 1
done
echo rc=$?
