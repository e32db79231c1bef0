#!/bin/bash
# Round 5: the 16-bit weight gradient's chunk ring (LDM_WGRAD_RING 2 / 3 / 4): bitwise tests, per-layer timing
set -o pipefail
OUT=gpurun_out/${1:-wgring}
mkdir -p $OUT
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
for shp in "256 4 16 512 3 2" "32 16 64 64 3 1" "512 2 8 256 3 2 T"; do
  timeout -k 10 60 python tools/one_conv.py wgrad $shp --maps32 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python $GRAFT_REPO_ROOT/tools/one_conv.py wgrad 256 4 16 512 3 2 --maps32 > /dev/null 2>&1 || exit 1
python - <<PY
import csv, glob
for f in glob.glob("$GRAFT_REPO_ROOT/$OUT/prof/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:90], r["Calls"], r["AverageNs"])
PY
