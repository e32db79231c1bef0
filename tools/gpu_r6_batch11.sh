#!/bin/bash
# Round 6, batch 11: the Cin = 1 k3 stride-1 conv on conv_cin1_x4_kernel (SD = 1; UNet(1, 1)'s first layer at
# shape S): the bitwise test against conv_cin1_kernel, the conv / store16 suites, then the stress line with
# LDM_CIN1_S1=0 / 1, twice around, and a kernel summary of the new default.   bash tools/gpu_r6_batch11.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b11}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_store16.py tests/test_gpu_parity.py tests/test_gpu_shape_s.py tests/test_gpu_cout1.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $OUT/tests.log | head; echo "tests exited $rc: stopping"; exit $rc; fi
for r in 1 2; do
  for m in 0 1; do
    LDM_CIN1_S1=$m timeout -k 10 240 python -u bench.py --workload stress --steps 3 --warmup 1 --no-cpu-baseline \
        > $OUT/stress_${r}_$m.json 2> $OUT/stress.err || { tail -20 $OUT/stress.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/stress_${r}_$m.json')); print('round $r cin1_s1=$m', d['us_per_denoise_iteration'], 'us/iter')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress.log; exit 1; }
echo done
