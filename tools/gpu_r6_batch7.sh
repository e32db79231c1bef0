#!/bin/bash
# Round 6, batch 7: the "wide" step-kernel variant (uconv.hip kKs3: 16 waves per block, one channel chunk per wave;
# enc4 without a K split, dec4 split over 2 blocks), parity first (the step-kernel and bench-config suites under
# LDM_UCONV_KS3=0x28), then the fp32 and fp16 loops per mask, twice around.   bash tools/gpu_r6_batch7.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b7}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
LDM_UCONV_KS3=0x28 timeout -k 10 400 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests_ks3.log 2>&1
rc=$?; tail -2 $OUT/tests_ks3.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests_ks3.log | head; echo "ks3 tests exited $rc: stopping"; exit $rc; fi
for r in 1 2; do
  for m in 0 0x08 0x20 0x28; do
    LDM_UCONV_KS3=$m timeout -k 10 120 python -u tools/loop_times.py > $OUT/loop_${r}_$m.txt 2>&1 || { tail $OUT/loop_${r}_$m.txt; exit 1; }
    echo "round $r ks3=$m: $(grep loop $OUT/loop_${r}_$m.txt)"
  done
  for m in 0 0x28; do
    LDM_UCONV_KS3=$m timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing \
        > $OUT/transfer_${r}_$m.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/transfer_${r}_$m.json')); print('round $r transfer ks3=$m', d['us_per_denoise_iteration'], 'us/iter')"
  done
done
LDM_UCONV_KS3=0x28 timeout -k 10 120 python -u tools/step_times.py --no-loop --layers 3,5 > $OUT/layers_ks3.txt 2>&1 && cat $OUT/layers_ks3.txt
timeout -k 10 120 python -u tools/step_times.py --no-loop --layers 3,5 > $OUT/layers_base.txt 2>&1 && cat $OUT/layers_base.txt
# flash attention forward with two key groups per block (LDM_FLASH_KH): parity under both forms, then the stress line
LDM_FLASH_KH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_attention_wide.py tests/test_gpu_shape_s.py -q -x \
    --timeout 240 --timeout-method thread > $OUT/tests_kh1.log 2>&1 || { tail -30 $OUT/tests_kh1.log; exit 1; }
tail -1 $OUT/tests_kh1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention_wide.py tests/test_gpu_shape_s.py -q -x \
    --timeout 240 --timeout-method thread > $OUT/tests_kh.log 2>&1 || { tail -30 $OUT/tests_kh.log; exit 1; }
tail -1 $OUT/tests_kh.log
for kh in 1 0; do
  LDM_FLASH_KH=$kh timeout -k 10 300 python -u bench.py --workload stress --steps 3 --warmup 1 --no-cpu-baseline > $OUT/stress_kh$kh.json 2> $OUT/stress.err \
      || { tail -20 $OUT/stress.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/stress_kh$kh.json')); print('stress kh=$kh', d['us_per_denoise_iteration'], 'us/iter', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_train_mc -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_train_mc.log 2>&1 \
    || { echo "rocprof train (memory copies) failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_train_mc.log; exit 1; }
echo done
