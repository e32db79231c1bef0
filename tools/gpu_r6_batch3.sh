#!/bin/bash
# Round 6, batch 3: the whole -m gpu suite (test failures are recorded, a fault / abort / timeout ends the call),
# then: the 16-bit (config 5) loop under K-split choices; the fp32 loop with dec4 slab-free and dec4's PMC traffic
# in that form; the train step with 1 / 2 / 4 pieces in flight in the BatchNorm sweeps; the stress line (flash
# attention double-buffered) with its rocprofv3 summary; rocprofv3 summaries of the transfer and train lines.
#   bash tools/gpu_r6_batch3.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b3}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest -m gpu exited $rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
tr() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > $OUT/transfer_$tag.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/transfer_$tag.json')); print('transfer $tag', d['us_per_denoise_iteration'], 'us/iter')"
}
sm() {
  local tag=$1; shift
  env "$@" timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
      > $OUT/sample_$tag.json 2> $OUT/sample.err || { tail -20 $OUT/sample.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/sample_$tag.json')); print('sample $tag', d['us_per_denoise_iteration'], 'us/iter')"
}
trn() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/train_$tag.json 2> $OUT/train.err || { tail -20 $OUT/train.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/train_$tag.json')); print('train $tag', round(d['ms_per_step'],4), 'ms')"
}
tr base || exit 1
tr ks0 LDM_UCONV_KS=0 || exit 1
tr ks10 LDM_UCONV_KS=0x10 || exit 1
tr ks18 LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 || exit 1
tr ks38v1 LDM_UCONV_KS=0x38 LDM_UCONV_KS2=0 || exit 1
tr ks7c LDM_UCONV_KS=0x7c || exit 1
sm base || exit 1
sm dec4nosplit LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 || exit 1
for r in 1 2; do
  trn u1_$r LDM_BN_UNROLL=1 || exit 1
  trn u2_$r LDM_BN_UNROLL=2 || exit 1
  trn u4_$r LDM_BN_UNROLL=4 || exit 1
done
timeout -k 10 300 python -u bench.py --workload stress --steps 3 --warmup 1 > $OUT/stress.json 2> $OUT/stress.err \
    || { tail -20 $OUT/stress.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/stress.json')); print('stress', d['us_per_denoise_iteration'], 'us/iter', d.get('roofline'))"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/$OUT/pmc_dec4ns_$C -o p -- \
      python3 $R/tools/step_times.py --no-loop --layers 5 --reps 20 > $R/$OUT/pmc_dec4ns_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $R/$OUT/pmc_dec4ns_$C.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_stress -o run -- \
    python3 $R/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $R/$OUT/prof_stress.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_transfer -o run -- \
    python3 $R/bench.py --workload transfer --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_transfer.log 2>&1 \
    || { echo "rocprof transfer failed"; tail $R/$OUT/prof_transfer.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_train -o run -- \
    python3 $R/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_train.log 2>&1 \
    || { echo "rocprof train failed"; tail $R/$OUT/prof_train.log; exit 1; }
echo done
