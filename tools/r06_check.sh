#!/bin/bash
# Round-6 GPU check: the GPU suite, smoke, the bench line and the per-op C2 table
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06a}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 python3 tools/fwd_ops.py > $O/fwd_ops_c2.txt 2>&1 &&
timeout -k 10 700 python3 -u bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log > $O/bench_line.json
echo rc=$?
