#!/bin/bash
# A/B timing of reverse-loop variants on the GPU box (replaces round 3's per-experiment gpu_r3_*.sh scripts).
#
#   bash tools/gpu_ab.sh <tag> [tests] <env-settings...>
#
# 1. optional parity gate ("tests" as the second argument): the step-kernel and bench-config suites under EVERY
#    env setting given (an A/B variant must be correct before it is timed);
# 2. the loop time per denoising iteration (tools/loop_times.py: config 2, B = 8, 16 x 64, graph replay) once per
#    setting, in the order given, twice around (boxes differ by 1-2 %: compare within one call only).
# Each setting is one word of space-free VAR=VALUE pairs joined by commas, e.g.
#   bash tools/gpu_ab.sh ks tests LDM_X=0 LDM_UCONV_KS=0x38,LDM_UCONV_KS2=0x28 LDM_UCONV_ENC3_THIN=1
# Output: gpurun_out/<tag>/loop_<i>.txt and one summary line per setting.  The round-3 experiments this covers
# (profiles/r03/README.md): K-split masks (LDM_UCONV_KS / _KS2), step geometries (LDM_UCONV_ENC2_WIDE,
# _ENC3_THIN, _DEC1_THIN), tap windows (LDM_UCONV_WINDOW / _PLANE).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
if [ "$1" = tests ]; then
  shift
  for s in "$@"; do
    env ${s//,/ } timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py \
      -x -q --timeout 240 --timeout-method thread > $O/tests_${s//[^A-Za-z0-9]/_}.log 2>&1
    rc=$?; echo "[$s] tests: $(tail -1 $O/tests_${s//[^A-Za-z0-9]/_}.log)"
    [ $rc -eq 0 ] || exit $rc
  done
fi
for rnd in 1 2; do
  i=0
  for s in "$@"; do
    i=$((i+1))
    env ${s//,/ } timeout -k 10 120 python -u tools/loop_times.py > $O/loop_${rnd}_$i.txt 2>&1 || { tail $O/loop_${rnd}_$i.txt; exit 1; }
    echo "round $rnd [$s]: $(grep loop $O/loop_${rnd}_$i.txt)"
  done
done
