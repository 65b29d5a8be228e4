#!/bin/bash
# C2 bench line under run-time kernel-choice knobs (no rebuild), two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs
mkdir -p $O
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --no-train --no-nms --no-predict --no-cpu-baseline --r50-batch 0 > $O/$n.log 2>&1 || return 1
  python3 -c "import json,sys; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['roofline']['frac'],4), round(d['roofline']['conv_ms_per_step'],3))" >> $O/summary.txt
}
for r in 1 2; do
  run base_$r X=1 && run tm1_$r JABD_M32_TM=1 && run tm2_$r JABD_M32_TM=2 && run kp2_$r JABD_EXPDW_KP=2 && run nw8_$r JABD_EXPDW_NW=8 || exit 1
done
echo rc=$?
