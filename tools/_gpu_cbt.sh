set -o pipefail
cd $GRAFT_REPO_ROOT
for tm in 4 2 1; do
JABD_CONV_TM=$tm JABD_CONV32=0 timeout -k 10 300 python -u tools/convbench.py --set mnv3 > gpurun_out/cbt$tm.txt 2>&1 || exit 1
done
echo ok
