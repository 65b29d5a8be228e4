#!/bin/bash
# Round-6 evidence at HEAD: kernel traces + rooflines (part B), then the
# counters (C4 PMC traffic, expdw SQ), then the conv-stack PMC + bench line (part A)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p profiles/r06
bash tools/r06_profile_b.sh > gpurun_out/r06_b.log 2>&1 && grep -q "rc=0" gpurun_out/r06_b.log &&
cp gpurun_out/r06/c4_step_roofline.json profiles/r06/ &&
bash tools/r06_pmc.sh > gpurun_out/r06_pmc.log 2>&1 && grep -q "rc=0" gpurun_out/r06_pmc.log &&
bash tools/r06_profile_a.sh > gpurun_out/r06_a.log 2>&1 && grep -q "rc=0" gpurun_out/r06_a.log
echo rc=$?
