set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch2 -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write2 -o run -- python3 bench.py --steps 3 --pmc-forward-only > $O/pmc_write.log 2>&1 &&
python3 tools/pmc_traffic.py $O/pmc_fetch2 $O/pmc_write2 3 $O/pmc_traffic.json
echo rc=$?
