#!/bin/bash
# Build a libjabd variant whose nms.o is compiled with extra flags:
#   tools/nms_variant.sh NAME "<flags>"  ->  abx/libjabd_NAME.so
# (A/B timing: JABD_LIB=abx/libjabd_NAME.so python3 tools/nms_steps.py)
set -e
cd "$(dirname "$0")/.."
CS=jabd-joint-attention-based-detector-for-small-face-detection_amd/csrc
mkdir -p abx
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -Wno-unused-variable -Iinclude -ffp-contract=off $2 -c $CS/nms.hip -o abx/nms_$1.o
objs=$(ls $CS/build/*.o | grep -v '/nms.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs abx/nms_$1.o -o abx/libjabd_$1.so \
  -Wl,-rpath,/opt/rocm/lib
