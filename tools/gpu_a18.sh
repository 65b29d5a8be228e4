set -o pipefail
O=gpurun_out/a18; mkdir -p $O
timeout -k 10 150 python3 -u tools/graph_check.py --no-detect --limit 120 > $O/g1.log 2>&1 || { echo G1FAIL; tail -30 $O/g1.log; exit 1; }
timeout -k 10 150 python3 -u tools/graph_check.py --limit 120 > $O/g2.log 2>&1 || { echo G2FAIL; tail -40 $O/g2.log; exit 1; }
echo ALLOK
