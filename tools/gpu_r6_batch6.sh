#!/bin/bash
# Round 6, batch 6: the whole -m gpu suite, then the train step (deferred bias-gradient finalizes incl. the BN dx sums, losses read back without a per-step host wait)
# (LDM_AMD_DEFER_BIAS), twice around, and a train rocprofv3 summary.   bash tools/gpu_r6_batch6.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b6}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest -m gpu exited $rc: stopping"; exit $rc; fi
trn() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/train_$tag.json 2> $OUT/train.err || { tail -20 $OUT/train.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/train_$tag.json')); print('train $tag', round(d['ms_per_step'],4), 'ms')"
}
for r in 1 2 3; do
  trn defer0_$r LDM_AMD_DEFER_BIAS=0 || exit 1
  trn defer1_$r LDM_AMD_DEFER_BIAS=1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_train -o run -- \
    python3 $R/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_train.log 2>&1 \
    || { echo "rocprof train failed"; tail $R/$OUT/prof_train.log; exit 1; }
echo done
