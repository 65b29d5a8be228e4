# C4 training-step HBM traffic by PMC (two passes) -> profiles/r05/pmc_traffic_c4.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05
T=/tmp/pmc_c4
mkdir -p $O $T profiles/r05
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/f -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2 > $O/pmc_c4_f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/w -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2 > $O/pmc_c4_w.log 2>&1 &&
python3 tools/pmc_train.py $T/f $T/w --steps 3 --roof profiles/r04/c4_step_roofline.json --out $O/pmc_traffic_c4.json > $O/pmc_c4_summary.txt &&
cp $O/pmc_traffic_c4.json profiles/r05/ && echo PMCOK
