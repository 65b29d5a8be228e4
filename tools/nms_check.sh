# NMS parity + timing on the GPU box: the NMS tests, then the C5 kernel stats
set -e
mkdir -p gpurun_out/nms12
timeout -k 10 300 python -u -m pytest tests/test_box_ops.py -k nms -x -q --timeout 240 --timeout-method thread > gpurun_out/nms12/t.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nms12/prof -o run -- python3 tools/nms_steps.py --reps 5 > gpurun_out/nms12/b.log 2>&1
