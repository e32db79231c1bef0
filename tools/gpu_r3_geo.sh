#!/bin/bash
# Round 3: step-layer geometry variants — parity, then loop times per env setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-geo}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
LDM_UCONV_ENC2_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/tests_enc2.log 2>&1
rc=$?; tail -2 $O/tests_enc2.log
if [ $rc -ne 0 ]; then echo "FAILED: enc2-wide tests rc=$rc"; exit $rc; fi
i=0
while read -r envs; do
  i=$((i+1))
  env $envs timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_$i.txt 2>&1 || exit 1
  echo "[$envs]: $(grep pairs $O/loop_$i.txt)"
done <<'LIST'
LDM_X=0
LDM_UCONV_ENC2_WIDE=1
LDM_UCONV_KS2=0x28
LDM_X=1
LIST
