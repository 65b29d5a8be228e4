set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr_r50b -o run -- python3 tools/train_steps.py --kind r50 --batch 64 --steps 2 > gpurun_out/tr_r50.log 2>&1; echo rc=$?; tail -2 gpurun_out/tr_r50.log
