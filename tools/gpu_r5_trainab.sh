#!/bin/bash
# Round 5: train-step A/B over environment settings (two bench runs each, alternating), after the train tests.
#   bash tools/gpu_r5_trainab.sh <tag> "ENV=a" "ENV=b" ...      ("-" = the defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/$1
shift
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py \
      tests/test_gpu_train_config3.py tests/test_gpu_train_fp16.py tests/test_gpu_config4_rank.py tests/test_gpu_store16.py \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for round in 1 2; do
  for setting in "$@"; do
    [ "$setting" = "-" ] && e="" || e="$setting"
    env $e timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
        > $O/train_${round}.json 2> $O/train.err || { echo "train failed ($setting)"; tail -20 $O/train.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/train_${round}.json')); print('$setting', round(d['ms_per_step'],4), 'ms', d.get('peak_mem_gb', ''))"
  done
done
