#!/bin/bash
# Round-6 final check at HEAD: GPU suite, smoke, C2 per-op table, bench line, then the C3
# kernel trace + step roofline (the R50 GEMM / bn3 changes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f
T=/tmp/prof_r06f
mkdir -p $O $T
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 python3 tools/fwd_ops.py > $O/fwd_ops_c2.txt 2>&1 &&
timeout -k 10 700 python3 -u bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log > $O/bench_line.json &&
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d $T/prof_tr_r50 -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/tr_r50.log 2>&1 &&
python3 tools/prof_summary.py $T/prof_tr_r50 --csv $O/kernel_stats_c3_r50_train.csv > $O/summary_c3_r50_train.txt &&
timeout -k 10 300 python3 tools/train_roofline.py --kind r50 --batch 64 --out $O/c3_step_roofline.json > $O/c3_step_roofline.txt 2>&1
echo rc=$?
