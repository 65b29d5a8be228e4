set -e
mkdir -p gpurun_out/nms1
for v in base noiou nostore; do
  if [ $v = base ]; then L=""; else L=abx/libjabd_$v.so; fi
  JABD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nms1/$v -o run -- python3 tools/nms_steps.py --reps 5 > gpurun_out/nms1/$v.log 2>&1
done
JABD_LIB=abx/libjabd_trace.so timeout -k 10 120 python3 tools/nms_steps.py --reps 1 > gpurun_out/nms1/trace.log 2>&1
