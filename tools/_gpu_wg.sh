set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1; do
JABD_WGRAD32=$v timeout -k 10 300 python -u tools/wgradbench.py > gpurun_out/wg_$v.txt 2>&1 || exit 1
done
echo ok
