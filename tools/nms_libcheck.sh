# NMS C5 bit-exactness + timing with an alternative build: bash tools/nms_libcheck.sh NAME
# (a failing assertion is recorded and the timing still runs; a crash or a
# time limit ends the script)
set -e
mkdir -p gpurun_out/nmsl
rc=0
JABD_LIB=abx/libjabd_$1.so timeout -k 10 300 python -u -m pytest tests/test_box_ops.py -k nms -x -q --timeout 240 --timeout-method thread > gpurun_out/nmsl/t_$1.log 2>&1 || rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
JABD_LIB=abx/libjabd_$1.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nmsl/prof_$1 -o run -- python3 tools/nms_steps.py --reps 5 > gpurun_out/nmsl/b_$1.log 2>&1
