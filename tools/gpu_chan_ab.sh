#!/bin/bash
# Channel-block activation backward (LDM_ACT_BWD_CHAN): parity, then the train-step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_store16.py tests/test_gpu_train_config3.py tests/test_gpu_amp.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
bash tools/gpu_train_ab.sh $T/ab LDM_ACT_BWD_CHAN=1 LDM_ACT_BWD_CHAN=0
