#!/bin/bash
# Round 6: the fp32-map weight-gradient ring (wgrad_lpp_kernel) against the double-buffered form (LDM_WGRAD_RING=2),
# bitwise, then per-layer timing of the UNet-level weight gradients (fp32 maps), then the train-step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6wgpp}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad_ring32.py \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for ring in 2 3 4; do
  for shp in "64 16 64 128 3 2" "128 8 32 256 3 2" "256 4 16 512 3 2" "512 2 8 512 3 1" "32 16 64 64 3 1" "512 2 8 256 3 2 T"; do
    LDM_WGRAD_RING=$ring timeout -k 10 60 python tools/one_conv.py wgrad $shp --maps32 | sed "s/^/ring=$ring /" || exit 1
  done
done
