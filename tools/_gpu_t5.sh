set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/convbench.py --set mnv3 > gpurun_out/cb5.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-train > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
