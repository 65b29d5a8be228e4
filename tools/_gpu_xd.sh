set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/convbench.py --set xd > gpurun_out/xd.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_xd -o run -- python3 tools/convbench.py --set xd --only b2.xd,b3.xd,b12.xd --reps 2 > gpurun_out/pmc_xd.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_xd2 -o run -- python3 tools/convbench.py --set xd --only b2.xd,b3.xd,b12.xd --reps 2 > gpurun_out/pmc_xd2.log 2>&1
echo rc=$?
