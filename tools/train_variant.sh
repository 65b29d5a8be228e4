#!/bin/bash
# Build a libjabd variant whose train.o is compiled with extra flags:
#   tools/train_variant.sh NAME "<flags>"  ->  abx/libjabd_NAME.so
set -e
cd "$(dirname "$0")/.."
CS=jabd-joint-attention-based-detector-for-small-face-detection_amd/csrc
mkdir -p abx
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -Wno-unused-variable -Iinclude -ffp-contract=fast $2 -c $CS/train.hip -o abx/train_$1.o
objs=$(ls $CS/build/*.o | grep -v '/train.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs abx/train_$1.o -o abx/libjabd_$1.so \
  -Wl,-rpath,/opt/rocm/lib
