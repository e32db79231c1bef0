#!/bin/bash
# Round 5: the 16-tap window form on 128-row tiles (LDM_TCONV_WIN bit 4)
set -o pipefail
OUT=gpurun_out/${1:-k16}
mkdir -p $OUT
LDM_TCONV_WIN=27 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store16.py \
    tests/test_gpu_tiled.py tests/test_gpu_train_config3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for win in 11 27; do
  LDM_TCONV_WIN=$win timeout -k 10 60 python tools/one_conv.py dgrad 128 32 128 64 4 2 T | sed "s/^/win=$win /" || exit 1
  LDM_TCONV_WIN=$win timeout -k 10 60 python tools/one_conv.py fwd 64 64 256 128 4 2 | sed "s/^/win=$win /" || exit 1
done
for round in 1 2; do
  for win in 11 27; do
    LDM_TCONV_WIN=$win timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
        > $OUT/train.json 2> $OUT/train.err || { tail -20 $OUT/train.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/train.json')); print('win=$win', d['ms_per_step'])"
  done
done
