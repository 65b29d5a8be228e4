#!/bin/bash
# Round-6 counters at HEAD: C4 training-step HBM traffic per kernel family
# (two PMC passes; raw counter CSVs kept) and the expdw1 SQ counters on
# b1 / b3 (convbench b2.xd / b4.xd, the skip-branch forms the model runs;
# three passes) -> gpurun_out/r06/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06
T=/tmp/pmc_c4
mkdir -p $O $T
ROOF=profiles/r06/c4_step_roofline.json
[ -f $ROOF ] || ROOF=profiles/r05/c4_step_roofline.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/f -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2 > $O/pmc_c4_f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/w -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2 > $O/pmc_c4_w.log 2>&1 &&
mkdir -p $O/raw_c4_f $O/raw_c4_w && cp $(find $T/f -name '*counter_collection.csv') $O/raw_c4_f/ && cp $(find $T/w -name '*counter_collection.csv') $O/raw_c4_w/ &&
python3 tools/pmc_train.py $T/f $T/w --steps 3 --roof $ROOF --out $O/pmc_traffic_c4.json > $O/pmc_c4_summary.txt &&
XD_SKIP_BRANCH=1 bash tools/pmc_sq.sh b2.xd,b4.xd expdw1 xd > $O/sq.log 2>&1 && cp gpurun_out/xdpmc/summary.txt $O/pmc_sq_expdw_b1b3_skip.txt
echo rc=$?
