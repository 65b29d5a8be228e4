set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1; do
  JABD_CONV32=$v timeout -k 10 300 python -u tools/convbench.py --set all > gpurun_out/cb_$v.txt 2>&1 || exit 1
done
echo DONE
