#!/bin/bash
# Round 6, batch 8: the wide step-kernel variant on more layers (uconv.hip kKs3: enc1 bit 0, enc3 bit 2, dec3 bit 6,
# dec2 bit 7; enc4 / dec4 are on by default): parity under all of them, then the fp32 loop per mask (twice around)
# and the fp16 loop.   bash tools/gpu_r6_batch8.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b8}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
LDM_UCONV_KS3=0xED timeout -k 10 400 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests_ks3all.log 2>&1
rc=$?; tail -2 $OUT/tests_ks3all.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $OUT/tests_ks3all.log | head; echo "tests exited $rc: stopping"; exit $rc; fi
for r in 1 2; do
  for m in 0x28 0x29 0x2C 0x68 0xA8 0xED; do
    LDM_UCONV_KS3=$m timeout -k 10 120 python -u tools/loop_times.py > $OUT/loop_${r}_$m.txt 2>&1 || { tail $OUT/loop_${r}_$m.txt; exit 1; }
    echo "round $r ks3=$m: $(grep loop $OUT/loop_${r}_$m.txt)"
  done
done
for m in 0x28 0xED; do
  LDM_UCONV_KS3=$m timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > $OUT/transfer_$m.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/transfer_$m.json')); print('transfer ks3=$m', d['us_per_denoise_iteration'], 'us/iter')"
done
for m in 0x28 0xED; do
  LDM_UCONV_KS3=$m timeout -k 10 120 python -u tools/step_times.py --no-loop > $OUT/layers_$m.txt 2>&1 && cat $OUT/layers_$m.txt
done
echo done
