# A/B timing of NMS variant builds (tools/nms_variant.sh NAME FLAGS -> abx/libjabd_NAME.so)
set -e
mkdir -p gpurun_out/nmsab
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=abx/libjabd_$v.so; fi
  JABD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nmsab/$v -o run -- python3 tools/nms_steps.py --reps 5 > gpurun_out/nmsab/$v.log 2>&1
done
