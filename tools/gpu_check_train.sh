#!/bin/bash
# Parity of the conv paths the train step takes (tiled / VALU convs, autocast, config 3, train) and then the
# train-step A/B (tools/gpu_train_ab.sh) for the given settings.   bash tools/gpu_check_train.sh <tag> <settings...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_amp.py tests/test_gpu_train_config3.py \
  tests/test_gpu_train.py tests/test_gpu_parity.py tests/test_gpu_reference_shapes.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/tests.log | head -20; exit $rc; }
bash tools/gpu_train_ab.sh $T/ab "$@"
