# Round-6 profile, part A: conv-stack PMC traffic passes, then the bench line
set -o pipefail
R=${R:-r06}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$R
T=/tmp/prof_$R
mkdir -p $O $T profiles/$R
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/pmc_write -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_write.log 2>&1 &&
python3 tools/pmc_traffic.py $T/pmc_fetch $T/pmc_write 3 $O/pmc_traffic.json &&
cp $O/pmc_traffic.json profiles/$R/pmc_traffic.json &&
timeout -k 10 700 python -u bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log > $O/bench_line.json
echo rc=$?
