# depthwise wgrad: parity tests + C4-shape timing of the row-walking vs strip kernel
set -e
mkdir -p gpurun_out/dwwg
timeout -k 10 300 python -u -m pytest tests/test_train_ops.py -k "dwconvfn_grads or dw_bnin" -x -q --timeout 240 --timeout-method thread > gpurun_out/dwwg/t.log 2>&1
timeout -k 10 120 python3 tools/dwwg_bench.py > gpurun_out/dwwg/b.log 2>&1
JABD_DW_WGRAD_ROWS=0 timeout -k 10 120 python3 tools/dwwg_bench.py > gpurun_out/dwwg/b0.log 2>&1
