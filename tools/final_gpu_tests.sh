#!/bin/bash
# the full GPU suite and smoke on the committed build
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/final/gpu_tests2.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
