# depthwise training kernels: parity tests + C4-shape timing of the row walkers vs the strip kernels
set -e
mkdir -p gpurun_out/dw
timeout -k 10 300 python -u -m pytest tests/test_train_ops.py -k "dwconvfn_grads or dw_bnin or dw_fwd_bn_stats or nlm" -x -q --timeout 240 --timeout-method thread > gpurun_out/dw/t.log 2>&1
JABD_DW_ROWS=0 timeout -k 10 120 python3 tools/dwfwd_bench.py --save /tmp/dwref.pt > gpurun_out/dw/f0.log 2>&1
timeout -k 10 120 python3 tools/dwfwd_bench.py --ref /tmp/dwref.pt > gpurun_out/dw/f1.log 2>&1
timeout -k 10 400 python3 tools/train_roofline.py --kind mnv3 --batch 32 --out gpurun_out/dw/c4.json > gpurun_out/dw/c4.txt 2>&1
