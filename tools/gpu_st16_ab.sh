#!/bin/bash
# 16-bit storage A/B after a change to its kernels: the storage tests, then the train step with / without.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_store16.py -x -q --timeout 240 --timeout-method thread > $O/store16.log 2>&1
rc=$?; tail -1 $O/store16.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/store16.log | head -30; exit $rc; }
bash tools/gpu_train_ab.sh $T/ab LDM_AMD_STORE16=1 LDM_AMD_STORE16=0
