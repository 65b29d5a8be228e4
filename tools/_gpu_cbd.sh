set -o pipefail
cd $GRAFT_REPO_ROOT
for d in 0 1 2 3; do
CONV_DBG=$d JABD_CONV32=0 timeout -k 10 300 python -u tools/convbench.py --set mnv3 --only b1.proj,b2.proj,b3.proj,b5.proj,b8.proj,fpn.lat1 > gpurun_out/cbd$d.txt 2>&1 || exit 1
done
echo ok
