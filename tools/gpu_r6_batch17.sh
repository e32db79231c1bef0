#!/bin/bash
# Round 6, batch 17: the flash splits' workspace in per-stream lanes: the width-general attention suite (the engine's
# token-major merge included), the shape-S tests, the stress line (its captured loop must keep the splits) and its
# kernel summary.   bash tools/gpu_r6_batch17.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b17}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention_wide.py tests/test_gpu_shape_s.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error|assert" $OUT/tests.log | head -20; echo "tests exited $rc: stopping"; exit $rc; fi
timeout -k 10 240 python -u bench.py --workload stress --steps 3 --warmup 1 --no-cpu-baseline > $OUT/stress.json 2> $OUT/stress.err \
    || { tail -20 $OUT/stress.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/stress.json')); print('stress', d['us_per_denoise_iteration'], 'us/iter')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress.log; exit 1; }
echo done
