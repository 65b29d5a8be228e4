#!/bin/bash
# wgrad32 double-buffered 1x1 A/B: parity tests, wgradbench, C3 / C4 steps
# (in-tree vs abx/libjabd_old.so, interleaved)
set -o pipefail
mkdir -p gpurun_out/wgdb
timeout -k 10 400 python3 -u -m pytest tests/test_train_ops.py tests/test_modules.py tests/test_train_size.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/wgdb/t.log 2>&1 &&
JABD_LIB=abx/libjabd_old.so timeout -k 10 200 python3 -u tools/wgradbench.py > gpurun_out/wgdb/wb_old.log 2>&1 &&
timeout -k 10 200 python3 -u tools/wgradbench.py > gpurun_out/wgdb/wb_new.log 2>&1 &&
for v in old new old new; do
  if [ $v = old ]; then L=abx/libjabd_old.so; else L=; fi
  JABD_LIB=$L timeout -k 10 300 python3 tools/train_steps.py --kind r50 --batch 64 --steps 4 >> gpurun_out/wgdb/c3_$v.log 2>&1 || exit 1
  JABD_LIB=$L timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 >> gpurun_out/wgdb/c4_$v.log 2>&1 || exit 1
done
