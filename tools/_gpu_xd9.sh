set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/pmc_xdv2 -o run -- python3 tools/convbench.py --set xd --only b2.xd,b3.xd,b12.xd --reps 2 > gpurun_out/pmc_xdv2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_xdv2b -o run -- python3 tools/convbench.py --set xd --only b2.xd,b3.xd,b12.xd --reps 2 > gpurun_out/pmc_xdv2b.log 2>&1
echo rc=$?
