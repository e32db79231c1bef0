#!/bin/bash
# Round 6, batch 10: the wide form of enc2 (uconv.hip kKs3 bit 1): parity (step kernels,
# bench config, the step loop against the general loop) under LDM_UCONV_KS3=0x1EF, then the fp32 / fp16 loops against
# the default 0x1ED, twice around.   bash tools/gpu_r6_batch10.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b10}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
LDM_UCONV_KS3=0x1EF timeout -k 10 400 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests_dec1.log 2>&1
rc=$?; tail -2 $OUT/tests_dec1.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $OUT/tests_dec1.log | head; echo "tests exited $rc: stopping"; exit $rc; fi
for r in 1 2; do
  for m in 0x1ED 0x1EF; do
    LDM_UCONV_KS3=$m timeout -k 10 120 python -u tools/loop_times.py > $OUT/loop_${r}_$m.txt 2>&1 || { tail $OUT/loop_${r}_$m.txt; exit 1; }
    echo "round $r ks3=$m: $(grep loop $OUT/loop_${r}_$m.txt)"
    LDM_UCONV_KS3=$m timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing \
        > $OUT/transfer_${r}_$m.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/transfer_${r}_$m.json')); print('round $r transfer ks3=$m', d['us_per_denoise_iteration'], 'us/iter')"
  done
done
echo done
