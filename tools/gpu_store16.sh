#!/bin/bash
# 16-bit storage of the train step's large maps: kernel-level bitwise tests, the train-path parity suites,
# then the train-step A/B (LDM_AMD_STORE16=1 / 0) and a rocprofv3 summary per setting.   bash tools/gpu_store16.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_store16.py -x -v --timeout 240 --timeout-method thread > $O/store16.log 2>&1
rc=$?; tail -3 $O/store16.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/store16.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_config3.py tests/test_gpu_amp.py tests/test_gpu_dp_graph.py \
  tests/test_gpu_graph_state.py tests/test_gpu_tiled.py -x -q -s --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1
rc=$?; tail -3 $O/train_tests.log; grep -E "ref bf16-vs|ours vs" $O/train_tests.log | head -40
[ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/train_tests.log | head -30; exit $rc; }
bash tools/gpu_train_ab.sh $T/ab LDM_AMD_STORE16=1 LDM_AMD_STORE16=0 || exit 1
