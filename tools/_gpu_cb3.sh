set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1; do
JABD_CONV32=$v timeout -k 10 300 python -u tools/convbench.py --set r50 > gpurun_out/cb3_$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_train_ops.py tests/test_train.py tests/test_model.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; echo rc=$?; tail -3 gpurun_out/pt.log
