#!/bin/bash
# Build a libjabd variant whose expdw.o is compiled with extra flags (and
# optionally from another copy of expdw.hip):
#   tools/xd_variant.sh NAME "<flags>" [expdw source]  ->  abx/libjabd_NAME.so
# (A/B timing: JABD_LIB=abx/libjabd_NAME.so python3 tools/convbench.py --set xd)
set -e
cd "$(dirname "$0")/.."
CS=jabd-joint-attention-based-detector-for-small-face-detection_amd/csrc
mkdir -p abx
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -Wno-unused-variable -Iinclude -I$CS -ffp-contract=fast $2 -c ${3:-$CS/expdw.hip} -o abx/expdw_$1.o
objs=$(ls $CS/build/*.o | grep -v '/expdw.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs abx/expdw_$1.o -o abx/libjabd_$1.so \
  -Wl,-rpath,/opt/rocm/lib
