#!/bin/bash
# Side-stream forms of the train step (ldm_amd/graphs.py): parity of the train tests under the given settings,
# then the graphed train-step A/B (tools/gpu_train_ab.sh).   bash tools/gpu_branch_ab.sh <tag> <settings...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
for s in "$@"; do
  env ${s//,/ } timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_config3.py tests/test_gpu_dp_graph.py \
    tests/test_gpu_graph_state.py -x -q --timeout 300 --timeout-method thread > $O/tests_${s//[^A-Za-z0-9]/_}.log 2>&1
  rc=$?; echo "[$s] tests: $(tail -1 $O/tests_${s//[^A-Za-z0-9]/_}.log)"
  [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/tests_${s//[^A-Za-z0-9]/_}.log | head -20; exit $rc; }
done
bash tools/gpu_train_ab.sh $T/ab "$@"
