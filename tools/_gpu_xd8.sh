set -o pipefail
cd $GRAFT_REPO_ROOT
JABD_EXPDW_EC16=1 timeout -k 10 300 python -u tools/convbench.py --set xd > gpurun_out/xd_v2ec16.txt 2>&1
echo rc=$?
