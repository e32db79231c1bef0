#!/bin/bash
# Round 4 combined check: (1) the step kernels with the XCD-grid block order (parity, then loop time with and
# without it), (2) the train-step conv window forms (tools/gpu_r4_tconvw.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4combo}; O=$PWD/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -2 $O/step_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/step_tests.log | head; exit $rc; }
for rnd in 1 2; do
  for x in 1 0; do
    LDM_UCONV_XCD=$x timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_xcd${x}_$rnd.txt 2>&1 || { tail $O/loop_xcd${x}_$rnd.txt; exit 1; }
    echo "round $rnd LDM_UCONV_XCD=$x: $(grep pairs $O/loop_xcd${x}_$rnd.txt)"
  done
done
timeout -k 10 600 bash tools/pmc_step_traffic.sh gpurun_out/$T/pmc 0 1 2 3 4 5 6 7 > $O/pmc.log 2>&1 || { echo pmc failed; tail -5 $O/pmc.log; exit 1; }
grep -A10 per_launch_bytes $O/pmc/pmc_traffic_step.json | head -10
bash tools/gpu_r4_tconvw.sh $T/tcw
