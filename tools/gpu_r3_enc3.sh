#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-enc3}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py tests/test_gpu_step_pairs.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: step tests rc=$rc"; exit $rc; fi
for e in 1 0; do
  LDM_UCONV_ENC3_THIN=$e timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_thin$e.txt 2>&1 || exit 1
  echo "enc3 thin $e: $(grep pairs $O/loop_thin$e.txt)"
done
