#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, as MI355X_MICROARCH.md prescribes) over the dispatches
# of kernels matching a regex in a bench workload.   bash tools/pmc_kernel.sh <tag> <regex> <bench args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; RX=$2; shift 2
O=$PWD/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $O/p$i -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
