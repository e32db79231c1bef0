#!/bin/bash
# Round 6: the Cin = 1 conv's channel-pair packed form: bitwise test, per-layer timing, config-3 parity with it on,
# train-step A/B (LDM_CIN1_PK 0 / 1, two rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6cin1pk}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_store16.py -k "cin1" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for pk in 0 1; do
  LDM_CIN1_PK=$pk timeout -k 10 60 python tools/one_conv.py fwd 1 128 512 64 3 2 --x32 | sed "s/^/pk=$pk /" || exit 1
  LDM_CIN1_PK=$pk timeout -k 10 60 python tools/one_conv.py fwd 1 128 512 64 4 2 --x32 | sed "s/^/pk=$pk /" || exit 1
  LDM_CIN1_PK=$pk timeout -k 10 60 python tools/one_conv.py dgrad 64 64 256 1 4 2 T | sed "s/^/pk=$pk /" || exit 1
done
LDM_CIN1_PK=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_config3.py \
    tests/test_gpu_train_fp16.py > $OUT/tests_pk.log 2>&1 || { tail -40 $OUT/tests_pk.log; exit 1; }
tail -1 $OUT/tests_pk.log
for round in 1 2; do
  for pk in 0 1; do
    LDM_CIN1_PK=$pk timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
        > $OUT/train_${pk}_${round}.json 2> $OUT/train.err || { tail -20 $OUT/train.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/train_${pk}_${round}.json')); print('pk $pk', round(d['ms_per_step'],4), 'ms')"
  done
done
