#!/bin/bash
# A/B of the train step (config 3, B = 32 bf16, graph replay) over env settings (replaces round 4's per-experiment
# session scripts).
#
#   bash tools/gpu_train_ab.sh <tag> [tests] <settings...>
#
# 1. optional parity gate ("tests" as the second argument): the train-path suites (train step, config 3, 16-bit
#    storage, autocast, 1x1 weight gradient, graph state, DP graph) under EVERY setting given;
# 2. bench.py --workload train per setting, in the order given, twice around (boxes differ by a few per cent:
#    compare within one call only), then one rocprofv3 --kernel-trace --stats summary per setting.
# A setting is space-free VAR=VALUE pairs joined by commas, e.g.
#   bash tools/gpu_train_ab.sh st16 tests LDM_AMD_STORE16=1 LDM_AMD_STORE16=0
# Switches measured this way: LDM_AMD_STORE16, LDM_AMD_STORE16_MIN, LDM_AMD_BRANCH_STREAMS,
# LDM_WGRAD_1X1, LDM_TCONV_WIN, LDM_AMD_AUTOCAST_OUT, LDM_BN_BLOCKS, LDM_REDUCE_W8.
# Output: gpurun_out/<tag>/train_<round>_<i>.json, prof_<i>/ and one summary line per setting and round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
if [ "$1" = tests ]; then
  shift
  for s in "$@"; do
    n=${s//[^A-Za-z0-9]/_}
    env ${s//,/ } timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_config3.py \
      tests/test_gpu_store16.py tests/test_gpu_amp.py tests/test_gpu_wgrad1x1.py tests/test_gpu_graph_state.py \
      tests/test_gpu_dp_graph.py -x -q --timeout 300 --timeout-method thread > $O/tests_$n.log 2>&1
    rc=$?; echo "[$s] tests: $(tail -1 $O/tests_$n.log)"
    [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $O/tests_$n.log | head -20; exit $rc; }
  done
fi
for rnd in 1 2; do
  i=0
  for s in "$@"; do
    i=$((i+1))
    env ${s//,/ } timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_${rnd}_$i.json 2> $O/train_${rnd}_$i.err || { tail $O/train_${rnd}_$i.err; exit 1; }
    echo "round $rnd [$s]: $(python3 -c "import json; d=json.load(open('$O/train_${rnd}_$i.json')); print(d['ms_per_step'], 'ms')")"
  done
done
i=0
for s in "$@"; do
  i=$((i+1))
  env ${s//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$i.log 2>&1 || { echo "rocprof failed"; tail $O/prof_$i.log; exit 1; }
done
