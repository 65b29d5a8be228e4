set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr_mnv3 -o run -- python3 tools/train_steps.py --kind mnv3 > gpurun_out/tr_mnv3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr_r50 -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > gpurun_out/tr_r50.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fwd -o run -- python3 bench.py --steps 10 --pmc-forward-only > gpurun_out/prof_fwd.log 2>&1
echo rc=$?
