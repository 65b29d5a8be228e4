mkdir -p gpurun_out/dw3
JABD_DW_DGRAD_ROWS=0 timeout -k 10 300 python -u -m pytest tests/test_train_ops.py -k "dw_dgrad_bn_fused and bhw6" -q --timeout 240 --timeout-method thread > gpurun_out/dw3/t0.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_train_ops.py -k "dw_dgrad_bn_fused and bhw6" -q --timeout 240 --timeout-method thread > gpurun_out/dw3/t1.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
JABD_DW_DGRAD_ROWS=0 timeout -k 10 120 python3 tools/dwbwd_bench.py --save /tmp/dgref.pt > gpurun_out/dw3/b0.log 2>&1 &&
timeout -k 10 120 python3 tools/dwbwd_bench.py --ref /tmp/dgref.pt > gpurun_out/dw3/b1.log 2>&1
