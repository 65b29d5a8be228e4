set -e
mkdir -p gpurun_out/nmstr
JABD_LIB=abx/libjabd_trace.so timeout -k 10 120 python3 tools/nms_steps.py --reps 1 > gpurun_out/nmstr/trace.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_box_ops.py -k nms -x -q --timeout 240 --timeout-method thread > gpurun_out/nmstr/t.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nmstr/prof -o run -- python3 tools/nms_steps.py --reps 5 > gpurun_out/nmstr/b.log 2>&1
