set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CB_TORCH=1 JABD_CONV32=1 timeout -k 10 300 python -u tools/convbench.py --set all --only b12.proj,b15.exp,l1.c3,l3.c1,l4.c3 > gpurun_out/cb_torch.txt 2>&1 &&
for v in 0 1; do
JABD_CONV32=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_cb$v -o run -- python3 tools/convbench.py --only b12.proj,l3.c1 --set all --reps 3 > gpurun_out/pmc_cb$v.log 2>&1 || exit 1
done
echo DONE
