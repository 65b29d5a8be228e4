#!/bin/bash
# NLM kv+pool in one workgroup per image, single-pass apply: parity + C2 per-op table
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-nlm}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_model.py tests/test_train.py tests/test_modules.py tests/test_beca_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 150 python3 tools/fwd_ops.py > $O/fwd_ops_c2.txt 2>&1 &&
JABD_NLM_KVPOOL=0 timeout -k 10 150 python3 tools/fwd_ops.py > $O/fwd_ops_c2_kvpool0.txt 2>&1
echo rc=$?
