set -o pipefail
cd $GRAFT_REPO_ROOT
for tm in 0 1; do
JABD_M32_TM=$tm timeout -k 10 300 python -u tools/convbench.py --set all --only b11.proj,b12.proj,b12.exp,l1.c2,l1.c3,l2.c1,l2.c2,l2.c3,l3.c1,l3.c2,l3.c3,l4.c3 > gpurun_out/m32_$tm.txt 2>&1 || exit 1
done
echo ok
