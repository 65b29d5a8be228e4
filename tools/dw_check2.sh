# depthwise data gradient + BN backward: parity tests + row walker vs strip-row timing
set -e
mkdir -p gpurun_out/dw2
timeout -k 10 400 python -u -m pytest tests/test_train_ops.py -k "dw_dgrad_bn_fused or dwconvfn_grads or dw_bnin" -x -q --timeout 300 --timeout-method thread > gpurun_out/dw2/t.log 2>&1
JABD_DW_DGRAD_ROWS=0 timeout -k 10 120 python3 tools/dwbwd_bench.py --save /tmp/dgref.pt > gpurun_out/dw2/b0.log 2>&1
timeout -k 10 120 python3 tools/dwbwd_bench.py --ref /tmp/dgref.pt > gpurun_out/dw2/b1.log 2>&1
timeout -k 10 400 python3 tools/train_roofline.py --kind mnv3 --batch 32 --out gpurun_out/dw2/c4.json > gpurun_out/dw2/c4.txt 2>&1
