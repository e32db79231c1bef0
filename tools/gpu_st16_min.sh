#!/bin/bash
# The 16-bit storage threshold: config-3 parity and the train tests at LDM_AMD_STORE16_MIN=2^20, then the step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
LDM_AMD_STORE16_MIN=1048576 timeout -k 10 600 python -u -m pytest tests/test_gpu_train_config3.py tests/test_gpu_train.py -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "ref bf16-vs|ours vs" $O/tests.log | head -16; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
bash tools/gpu_train_ab.sh $T/ab LDM_AMD_STORE16_MIN=1048576 LDM_AMD_STORE16_MIN=4194304
