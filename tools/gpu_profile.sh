# Round profile: conv-stack HBM traffic PMC passes (MI355X_MICROARCH.md: one
# counter family per pass), then the bench line (which reads that traffic from
# profiles/<round>/pmc_traffic.json), then kernel-trace stats of the C2
# forward, the training steps and C5 NMS.  Raw rocprofv3 output stays in
# /tmp on the box; only logs and the per-kernel CSV summaries go to
# gpurun_out/<round>/ (the merge-back is capped at 64 MiB).
# Usage on the GPU box: bash tools/gpu_profile.sh r03
set -o pipefail
R=${1:-r02}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$R
T=/tmp/prof_$R
mkdir -p $O $T profiles/$R
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/pmc_write -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_write.log 2>&1 &&
python3 tools/pmc_traffic.py $T/pmc_fetch $T/pmc_write 3 $O/pmc_traffic.json &&
cp $O/pmc_traffic.json profiles/$R/pmc_traffic.json &&
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log > $O/bench_line.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_fwd -o run -- python3 bench.py --steps 10 --pmc-forward-only > $O/prof_fwd.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_tr_mnv3 -o run -- python3 tools/train_steps.py --kind mnv3 > $O/tr_mnv3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_tr_r50 -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > $O/tr_r50.log 2>&1 &&
timeout -k 10 200 python3 tools/fwd_ops.py > $O/fwd_ops_c2.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/prof_nms -o run -- python3 tools/nms_steps.py --reps 5 > $O/nms_steps.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_tr_beca -o run -- python3 tools/train_steps.py --kind beca --steps 2 > $O/tr_beca.log 2>&1 &&
for d in prof_fwd:c2_forward prof_tr_mnv3:c4_mnv3_train prof_tr_r50:c3_r50_train prof_nms:c5_nms prof_tr_beca:beca_train; do
  python3 tools/prof_summary.py $T/${d%%:*} --csv $O/kernel_stats_${d##*:}.csv > $O/summary_${d##*:}.txt || exit 1
done
echo rc=$?
