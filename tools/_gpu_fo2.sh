set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/fwd_ops.py > gpurun_out/fwd_ops_mnv3.txt 2>&1; echo rc=$?
