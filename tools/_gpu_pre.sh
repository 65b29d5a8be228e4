set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1; do
JABD_CONV_PRE=$v timeout -k 10 300 python -u tools/convbench.py --set mnv3 --only b2.proj,b3.proj,b4.proj,b5.proj,fpn.lat1 > gpurun_out/pre_$v.txt 2>&1 || exit 1
done
echo ok
