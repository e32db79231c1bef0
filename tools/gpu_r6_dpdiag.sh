#!/bin/bash
# Round 6: the data-parallel graphed-step tests alone, uncaptured output (-s) so a runtime / RCCL abort message is kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6dp}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_config4_rank.py \
    tests/test_gpu_dp_graph.py > $OUT/tests_dp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|rror|terminate|what\(\)|Abort" $OUT/tests_dp.log | head -30
exit $rc
