#!/bin/bash
# streaming 1x1 GEMM form + specialised epilogues: parity, bit-identity A/B, C3 step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/m32s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_ops.py tests/test_train_size.py -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model.py -m gpu -k "r50 or R50 or resnet" > $O/tests_model.log 2>&1 &&
JABD_M32S=1 timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/on > $O/on.log 2>&1 &&
JABD_M32S=0 timeout -k 10 200 python3 -u tools/m32s_ab.py --out $O/off > $O/off.log 2>&1 &&
python3 tools/m32s_ab.py --compare $O/on $O/off > $O/cmp.log 2>&1 &&
for i in 1 2; do
JABD_M32S=1 timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_on_$i.log 2>&1 &&
JABD_M32S=0 JABD_CONV32=0 timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_off_$i.log 2>&1 || exit 1
done
echo rc=$?
