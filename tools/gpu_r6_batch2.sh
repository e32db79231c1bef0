#!/bin/bash
# Round 6, batch 2: the whole -m gpu suite + smoke() on the new defaults, then the K-split choice of the 16-bit
# (config 5) loop and the slab-free dec4 form of the fp32 loop, each timed in the loop; dec4's PMC traffic in both
# forms; a rocprofv3 kernel summary of the fp16 transfer loop.   bash tools/gpu_r6_batch2.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b2}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
bash tools/gpu_r6_endA.sh $T || exit 1
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
tr base || exit 1
tr ks0 LDM_UCONV_KS=0 || exit 1
tr ks10 LDM_UCONV_KS=0x10 || exit 1
tr ks18 LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 || exit 1
tr ks38v1 LDM_UCONV_KS=0x38 LDM_UCONV_KS2=0 || exit 1
tr ks7c LDM_UCONV_KS=0x7c || exit 1
tr ks30 LDM_UCONV_KS=0x30 LDM_UCONV_KS2=0x20 || exit 1
sm base || exit 1
sm dec4nosplit LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 || exit 1
sm base2 || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  LDM_UCONV_KS=0x18 LDM_UCONV_KS2=0x08 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/$OUT/pmc_dec4ns_$C -o p -- \
      python3 $R/tools/step_times.py --no-loop --layers 5 --reps 20 > $R/$OUT/pmc_dec4ns_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $R/$OUT/pmc_dec4ns_$C.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_transfer -o run -- \
    python3 $R/bench.py --workload transfer --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_transfer.log 2>&1 \
    || { echo "rocprof transfer failed"; tail $R/$OUT/prof_transfer.log; exit 1; }
find $R/$OUT/prof_transfer -name "*stats*"
