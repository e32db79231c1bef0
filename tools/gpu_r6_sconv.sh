#!/bin/bash
# Round 6: plan kind 4 (sconv.hip): its tests, the train-path parity tests with it, per-call conv timings of the
# train step, then the train-step A/B (LDM_AMD_SCONV 0 / 1, two rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6sconv}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sconv.py \
    > $OUT/tests_sconv.log 2>&1 || { tail -40 $OUT/tests_sconv.log; exit 1; }
tail -1 $OUT/tests_sconv.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py \
    tests/test_gpu_train_config3.py tests/test_gpu_train_fp16.py tests/test_gpu_config4_rank.py tests/test_gpu_amp.py \
    tests/test_gpu_reference_shapes.py > $OUT/tests_train.log 2>&1 || { tail -40 $OUT/tests_train.log; exit 1; }
tail -1 $OUT/tests_train.log
timeout -k 10 300 python -u tools/train_conv_calls.py > $OUT/conv_calls.txt 2> $OUT/conv_calls.err || { tail -20 $OUT/conv_calls.err; exit 1; }
head -40 $OUT/conv_calls.txt
for round in 1 2; do
  for sc in 0 1; do
    LDM_AMD_SCONV=$sc timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
        > $OUT/train_${sc}_${round}.json 2> $OUT/train.err || { tail -20 $OUT/train.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/train_${sc}_${round}.json')); print('sconv $sc', round(d['ms_per_step'],4), 'ms')"
  done
done
