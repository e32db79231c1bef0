#!/bin/bash
# Full check of the tree: every -m gpu test, smoke(), the headline bench with its rocprofv3 summary, and the
# secondary lines (transfer, train + train kernel summary).   bash tools/gpu_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-round}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: pytest -m gpu exited $rc"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_final.sh ${1:-round}/final || exit 1
bash tools/gpu_workloads.sh ${1:-round}/workloads || exit 1
