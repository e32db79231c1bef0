#!/bin/bash
# Round 6: the weight-gradient chunk ring with its counted waits (no compiler drains): bitwise ring tests,
# per-layer timing for LDM_WGRAD_RING 2 / 3 / 4, then train-step A/B (two rounds, alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6wgring}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store16.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for ring in 2 3 4; do
  LDM_WGRAD_RING=$ring timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_store16.py -k ring > $OUT/tests_ring$ring.log 2>&1 || { tail -30 $OUT/tests_ring$ring.log; exit 1; }
  for shp in "128 32 128 64 4 2 T" "64 64 256 128 3 2" "128 32 128 256 3 2" "256 16 64 256 3 2" "128 32 128 32 3 2" \
             "64 64 256 1 4 2 T"; do
    LDM_WGRAD_RING=$ring timeout -k 10 60 python tools/one_conv.py wgrad $shp | sed "s/^/ring=$ring /" || exit 1
  done
done
if [ "${TRAIN:-1}" = 1 ]; then
  for round in 1 2; do
    for ring in 2 3 4; do
      LDM_WGRAD_RING=$ring timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
          > $OUT/train_${ring}_${round}.json 2> $OUT/train.err || { echo "train failed"; tail -20 $OUT/train.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/train_${ring}_${round}.json')); print('ring $ring', round(d['ms_per_step'],4), 'ms')"
    done
  done
fi
