set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fwd_ops.py > gpurun_out/fwd_ops_mnv3.txt 2>&1 &&
timeout -k 10 300 python -u tools/fwd_ops.py --kind r50 --batch 16 > gpurun_out/fwd_ops_r50.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fwd -o run -- python3 bench.py --steps 10 --pmc-forward-only > gpurun_out/prof_fwd.log 2>&1 && echo DONE
