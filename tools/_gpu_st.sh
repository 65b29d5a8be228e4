set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/fwd_ops.py > gpurun_out/fwd_ops_mnv3.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_model.py tests/test_train.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; echo rc=$?; tail -1 gpurun_out/pt.log
