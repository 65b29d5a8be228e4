set -o pipefail
cd $GRAFT_REPO_ROOT
JABD_EXPDW_V=3 timeout -k 10 300 python -u tools/convbench.py --set xd > gpurun_out/xd_v3.txt 2>&1 &&
JABD_EXPDW_V=2 timeout -k 10 300 python -u tools/convbench.py --set xd > gpurun_out/xd_v2.txt 2>&1
echo rc=$?
