#!/bin/bash
# Round 3: thin K-split variant (LDM_UCONV_KS2) — parity with it forced on, then loop times per mask pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-ks2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: step tests rc=$rc"; exit $rc; fi
for m in ${KSM:-0x38:0x38 0x18:0x00}; do
  LDM_UCONV_KS=${m%%:*} LDM_UCONV_KS2=${m##*:} timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_${m/:/_}.txt 2>&1 || exit 1
  echo "ks,ks2 $m: $(grep pairs $O/loop_${m/:/_}.txt)"
done
