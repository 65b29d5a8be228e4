set -e
mkdir -p gpurun_out/nmstr
JABD_LIB=abx/libjabd_trace.so timeout -k 10 120 python3 tools/nms_steps.py --reps 1 > gpurun_out/nmstr/trace.log 2>&1
