#!/bin/bash
# Round 5: tconvw 128-row wave grid (LDM_TCONVW_WNW 2 = 2 x 2, 1 = four waves along the rows)
set -o pipefail
OUT=gpurun_out/${1:-wnw}
mkdir -p $OUT
for wnw in 1 2; do
  LDM_TCONVW_WNW=$wnw timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store16.py \
      tests/test_gpu_tiled.py tests/test_gpu_train_config3.py > $OUT/tests$wnw.log 2>&1 || { tail -30 $OUT/tests$wnw.log; exit 1; }
  tail -1 $OUT/tests$wnw.log
done
for wnw in 1 2; do
  for shp in "fwd 64 64 256 128 3 2" "fwd 128 32 128 256 3 2" "fwd 256 16 64 256 3 2" "dgrad 256 16 64 256 3 2" \
             "fwd 256 8 32 128 3 2 T" "fwd 128 32 128 128 3 1"; do
    LDM_TCONVW_WNW=$wnw timeout -k 10 60 python tools/one_conv.py $shp | sed "s/^/wnw=$wnw /" || exit 1
  done
done
