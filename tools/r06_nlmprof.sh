#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-nlmprof}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p1 -o run -- python3 bench.py --steps 5 --pmc-forward-only > $O/p1.log 2>&1 &&
python3 tools/kernel_calls.py /tmp/p1 nlm eca_gate ssh_tail > $O/calls_kvpool1.txt &&
JABD_NLM_KVPOOL=0 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p0 -o run -- python3 bench.py --steps 5 --pmc-forward-only > $O/p0.log 2>&1 &&
python3 tools/kernel_calls.py /tmp/p0 nlm > $O/calls_kvpool0.txt
echo rc=$?
