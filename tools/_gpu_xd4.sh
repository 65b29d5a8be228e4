set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/convbench.py --set xd > gpurun_out/xd.txt 2>&1
echo rc=$?
