#!/bin/bash
# Round 6 end, part A: the whole -m gpu suite and smoke().   bash tools/gpu_r6_endA.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6end}; O=$PWD/gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; echo "FAILED: pytest -m gpu exited $rc"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
