# SQ issue/stall counters for the expand+depthwise kernels (three PMC passes,
# <= 8 SQ counters each), summarised per kernel by tools/pmc_kernel.py.
# Usage on the GPU box: bash tools/pmc_sq.sh [shapes] [kernel match] [convbench set]
#   (default b2.xd,b12.xd expdw1 xd)
set -o pipefail
SH=${1:-b2.xd,b12.xd}
MATCH=${2:-expdw1}
SET=${3:-xd}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/xdpmc
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 tools/convbench.py --set $SET --only $SH --reps 3 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_kernel.py $O/p1 $O/p2 $O/p3 --match $MATCH > $O/summary.txt
