#!/bin/bash
# SQ counters of the 1x1 32x32 GEMM on R50 l1.c3 (K 64 -> N 256): streaming form vs tile kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export JABD_CONV32=1
JABD_M32S=1 bash tools/pmc_sq.sh t.l1.c3 conv1x1_m32 r50t && mv gpurun_out/xdpmc gpurun_out/m32pmc_on &&
JABD_M32S=0 bash tools/pmc_sq.sh t.l1.c3 conv1x1_m32 r50t && mv gpurun_out/xdpmc gpurun_out/m32pmc_off
echo rc=$?
