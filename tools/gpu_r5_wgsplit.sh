#!/bin/bash
# Round 5: the weight gradient's K split cap (LDM_WGRAD_SPLITS) on the train step's layers (B = 32 bf16)
set -o pipefail
OUT=gpurun_out/${1:-wgsplit}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store16.py \
    tests/test_gpu_wgrad1x1.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cap in 256 64 16 4 1; do
  LDM_WGRAD_SPLITS=$cap timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_store16.py -k "ring or kind3" > $OUT/tests_cap$cap.log 2>&1 || { tail -30 $OUT/tests_cap$cap.log; exit 1; }
  for shp in "256 4 16 512 3 2 --maps32" "32 16 64 64 3 1 --maps32" "64 16 64 128 3 2 --maps32" "256 8 32 256 3 2 --maps32" \
             "512 2 8 512 3 1 --maps32" "128 32 128 64 4 2 T" "64 64 256 128 3 2" "256 16 64 256 3 2" "128 32 128 32 3 2"; do
    LDM_WGRAD_SPLITS=$cap timeout -k 10 60 python tools/one_conv.py wgrad $shp | sed "s/^/cap=$cap /" || exit 1
  done
done
