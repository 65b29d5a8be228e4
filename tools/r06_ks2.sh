#!/bin/bash
# which K = 64 GEMM forms the streaming kernel should take: C3 step per JABD_M32S_KS2 mask
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ks2
mkdir -p $O
for i in 1 2; do
  for m in 7 3 5 1; do
    JABD_M32S_KS2=$m timeout -k 10 200 python3 -u tools/train_steps.py --kind r50 --batch 64 --steps 6 > $O/c3_m${m}_$i.log 2>&1 || exit 1
  done
done
echo rc=$?
