set -o pipefail
cd $GRAFT_REPO_ROOT
for d in 0 3 7 11 19 27 31; do
XD_DBG=$d timeout -k 10 300 python -u tools/convbench.py --set xd --only b2.xd,b3.xd,b12.xd > gpurun_out/xd_dbg$d.txt 2>&1 || exit 1
done
echo ok
