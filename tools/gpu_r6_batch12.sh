#!/bin/bash
# Round 6, batch 12: the Cin = 1 conv's output channels split over grid.y at few pixel blocks (shape S), its tests,
# the stress line; then the shape-S conv plans autotuned (tools/tune_stress.py, merged into the box copy of
# tuned_plans.json and copied out), the shape-S tests and the stress line again on the tuned plans, and a kernel
# summary.   bash tools/gpu_r6_batch12.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b12}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_store16.py tests/test_gpu_shape_s.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $OUT/tests.log | head; echo "tests exited $rc: stopping"; exit $rc; fi
stress() {
  timeout -k 10 240 python -u bench.py --workload stress --steps 3 --warmup 1 --no-cpu-baseline > $OUT/stress_$1.json 2> $OUT/stress.err \
      || { tail -20 $OUT/stress.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/stress_$1.json')); print('$1', d['us_per_denoise_iteration'], 'us/iter')"
}
stress before_tune || exit 1
timeout -k 10 600 python -u tools/tune_stress.py --dump $OUT/tune_stress_times.json > $OUT/tune.log 2>&1 \
    || { tail -20 $OUT/tune.log; exit 1; }
grep -E "best|default|saved" $OUT/tune.log | tail -40
cp music-style-transfer-ldm_amd/tuned_plans.json $OUT/tuned_plans.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_shape_s.py -q -x --timeout 300 --timeout-method thread > $OUT/tests_tuned.log 2>&1
rc=$?; tail -2 $OUT/tests_tuned.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $OUT/tests_tuned.log | head; echo "tests exited $rc: stopping"; exit $rc; fi
stress tuned_1 && stress tuned_2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress.log; exit 1; }
echo done
