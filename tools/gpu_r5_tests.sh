#!/bin/bash
# A subset of -m gpu test files (arguments), then optional capture_wgrad repro cases (REPRO="case ...").
#   bash tools/gpu_r5_tests.sh <tag> tests/test_a.py tests/test_b.py::name ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
if [ -n "$REPRO" ]; then bash tools/gpu_capture_wgrad.sh $T/repro $REPRO || exit $?; fi
