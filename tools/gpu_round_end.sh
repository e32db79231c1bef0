#!/bin/bash
# Round-end validation: the whole -m gpu suite, smoke(), the headline bench with its rocprofv3 summary, the
# secondary lines (transfer, train + its kernel summary) and the train-step PMC passes, all under
# gpurun_out/<tag>/ (the judged copies go to profiles/rNN/ by hand).   bash tools/gpu_round_end.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-round_end}; O=$PWD/gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; echo "FAILED: pytest -m gpu exited $rc"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_final.sh $T/final || exit 1
bash tools/gpu_workloads.sh $T/workloads || exit 1
timeout -k 10 600 bash tools/pmc_train.sh gpurun_out/$T/pmc_train > $O/pmc_train.log 2>&1 || { echo "pmc_train failed"; tail $O/pmc_train.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/pmc_train/summary.json')); print('train HBM bytes/step', d.get('step_hbm_bytes'), 'mfma util', d.get('step_mfma_util'))"
