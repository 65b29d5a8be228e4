# Round-5 profile, part B: kernel-trace stats of the C2 forward, the C4 / C3
# training steps, C5 NMS, the per-op C2 forward table and the step rooflines
set -o pipefail
R=${R:-r06}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$R
T=/tmp/prof_$R
mkdir -p $O $T
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/prof_fwd -o run -- python3 bench.py --steps 10 --pmc-forward-only > $O/prof_fwd.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/prof_tr_mnv3 -o run -- python3 tools/train_steps.py --kind mnv3 > $O/tr_mnv3.log 2>&1 &&
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d $T/prof_tr_r50 -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/tr_r50.log 2>&1 &&
timeout -k 10 150 python3 tools/fwd_ops.py > $O/fwd_ops_c2.txt 2>&1 &&
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $T/prof_nms -o run -- python3 tools/nms_steps.py --reps 5 > $O/nms_steps.log 2>&1 &&
for d in prof_fwd:c2_forward prof_tr_mnv3:c4_mnv3_train prof_tr_r50:c3_r50_train prof_nms:c5_nms; do
  python3 tools/prof_summary.py $T/${d%%:*} --csv $O/kernel_stats_${d##*:}.csv > $O/summary_${d##*:}.txt || exit 1
done &&
timeout -k 10 300 python3 tools/train_roofline.py --kind mnv3 --batch 32 --out $O/c4_step_roofline.json > $O/c4_step_roofline.txt 2>&1 &&
timeout -k 10 300 python3 tools/train_roofline.py --kind r50 --batch 64 --out $O/c3_step_roofline.json > $O/c3_step_roofline.txt 2>&1
echo rc=$?
