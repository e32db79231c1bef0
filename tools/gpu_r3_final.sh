#!/bin/bash
# Round 3 final: step-kernel HBM traffic (PMC passes) for the bench's roofline, then the full round check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r3f}
bash tools/pmc_step_traffic.sh gpurun_out/$T/pmc 0 1 2 3 4 5 6 7 > gpurun_out/$T.pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/$T.pmc.log; exit 1; }
cp gpurun_out/$T/pmc/pmc_traffic_step.json profiles/r03/pmc_traffic_step.json
grep -A10 per_launch_bytes profiles/r03/pmc_traffic_step.json | head -12
bash tools/gpu_round.sh $T
