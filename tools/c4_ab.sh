# C4 step time A/B: bash tools/c4_ab.sh NAME... (abx/libjabd_NAME.so; "base" = the in-tree build)
set -e
mkdir -p gpurun_out/c4ab
i=0
for v in "$@"; do
  i=$((i+1))
  if [ $v = base ]; then L=""; else L=abx/libjabd_$v.so; fi
  JABD_LIB=$L timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 > gpurun_out/c4ab/${i}_$v.log 2>&1
done
