#!/bin/bash
# Round 4: the RCCL capture race (tools/dp_capture_repro.py) in thread-local mode, the DP-graph tests in-process
# over env://, the act-backward fix, the headline bench + rocprofv3 summary; LAST, the global-mode repro
# (expected to abort if the watchdog hypothesis holds: nothing runs after it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-r4dp}; mkdir -p $O
timeout -k 10 120 python -u tools/dp_capture_repro.py thread_local > $O/repro_tl.log 2>&1
echo "repro thread_local rc=$?"; tail -2 $O/repro_tl.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp_graph.py "tests/test_gpu_train.py::test_act_backward_none_separate_dv" \
  "tests/test_gpu_train.py::test_act_backward_sums" -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_final.sh ${1:-r4dp}/final || exit 1
TORCH_CPP_LOG_LEVEL=INFO timeout -k 10 120 python -u tools/dp_capture_repro.py global > $O/repro_global.log 2>&1
echo "repro global rc=$?"; tail -15 $O/repro_global.log
