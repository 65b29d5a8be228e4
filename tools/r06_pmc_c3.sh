#!/bin/bash
# C3 (R50 bs64 training step) HBM traffic per kernel family: two PMC passes (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06c3
T=/tmp/pmc_c3
mkdir -p $O $T
ROOF=profiles/r06/c3_step_roofline.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/f -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/pmc_c3_f.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/w -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/pmc_c3_w.log 2>&1 &&
python3 tools/pmc_train.py $T/f $T/w --steps 3 --roof $ROOF --out $O/pmc_traffic_c3.json > $O/pmc_c3_summary.txt
echo rc=$?
