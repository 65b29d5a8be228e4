# expdw3 phase-skip timing (results wrong; tools/convbench.py --set xd with XD_DBG)
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
for d in 0 1 2 4 6 8 16 32 63; do
  XD_DBG=$d timeout -k 10 120 python3 tools/convbench.py --set xd --only b1.xd,b2.xd,b3.xd,b4.xd,b5.xd,b7.xd --reps 10 > $O/dbg_$d.txt 2>&1 || { echo FAIL $d; tail -5 $O/dbg_$d.txt; exit 1; }
  echo "dbg=$d $(grep -E '^b' $O/dbg_$d.txt | awk '{printf "%s %s  ", $1, $6}')"
done
