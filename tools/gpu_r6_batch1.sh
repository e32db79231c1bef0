#!/bin/bash
# Round 6, one call: correctness of this round's kernels first (kind-4 sconv, fp32-map wgrad ring, Cin = 1 packed form,
# BN dx-sum), the train-path parity suite, then A/B timings (train step: sconv / dx-sum / cin1 packed; reverse loops:
# sub-batch chains), then a rocprofv3 summary of the train step.   bash tools/gpu_r6_batch1.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6b1}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sconv.py \
    tests/test_gpu_wgrad_ring32.py tests/test_gpu_store16.py > $OUT/tests_kernels.log 2>&1 || { tail -40 $OUT/tests_kernels.log; exit 1; }
tail -1 $OUT/tests_kernels.log
# (-s: nothing captured, so a runtime / RCCL abort message stays in the log)
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_config4_rank.py \
    tests/test_gpu_dp_graph.py tests/test_gpu_train.py tests/test_gpu_train_config3.py tests/test_gpu_train_fp16.py \
    tests/test_gpu_reference_shapes.py tests/test_gpu_graph_state.py tests/test_gpu_shape_s.py \
    > $OUT/tests_train.log 2>&1 || { grep -v "^  File" $OUT/tests_train.log | tail -40; exit 1; }
tail -1 $OUT/tests_train.log
LDM_CIN1_PK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_config3.py \
    > $OUT/tests_pk.log 2>&1 || { tail -30 $OUT/tests_pk.log; exit 1; }
tail -1 $OUT/tests_pk.log
for pk in 0 1; do
  LDM_CIN1_PK=$pk timeout -k 10 60 python tools/one_conv.py fwd 1 128 512 64 3 2 --x32 | sed "s/^/pk=$pk /" || exit 1
  LDM_CIN1_PK=$pk timeout -k 10 60 python tools/one_conv.py dgrad 64 64 256 1 4 2 T | sed "s/^/pk=$pk /" || exit 1
done
for ring in 2 3; do
  for shp in "64 16 64 128 3 2" "128 8 32 256 3 2" "256 4 16 512 3 2" "512 2 8 512 3 1"; do
    LDM_WGRAD_RING=$ring timeout -k 10 60 python tools/one_conv.py wgrad $shp --maps32 | sed "s/^/ring=$ring /" || exit 1
  done
done
run_train() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/train_$tag.json 2> $OUT/train.err || { tail -20 $OUT/train.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/train_$tag.json')); print('train $tag', round(d['ms_per_step'],4), 'ms')"
}
for round in 1 2; do
  run_train base_$round LDM_AMD_SCONV=0 LDM_AMD_BN_DXSUM=0 LDM_CIN1_PK=0 || exit 1
  run_train all_$round LDM_CIN1_PK=1 || exit 1
  run_train nopk_$round LDM_CIN1_PK=0 || exit 1
  run_train nosconv_$round LDM_AMD_SCONV=0 LDM_CIN1_PK=1 || exit 1
  run_train nodxsum_$round LDM_AMD_BN_DXSUM=0 LDM_CIN1_PK=1 || exit 1
  run_train noreduce4_$round LDM_WGRAD_REDUCE4=0 LDM_CIN1_PK=1 || exit 1
done
for sp in 1 2; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --split $sp --no-cpu-baseline --no-kernel-timing \
      > $OUT/sample_$sp.json 2> $OUT/sample.err || { tail -20 $OUT/sample.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/sample_$sp.json')); print('sample split $sp', d['us_per_denoise_iteration'], 'us/iter')"
  timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --split $sp --no-cpu-baseline --no-kernel-timing \
      > $OUT/transfer_$sp.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/transfer_$sp.json')); print('transfer split $sp', d['us_per_denoise_iteration'], 'us/iter')"
done
timeout -k 10 240 python -u bench.py --workload stress --steps 3 --warmup 1 > $OUT/stress.json 2> $OUT/stress.err \
    || { tail -20 $OUT/stress.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/stress.json')); print('stress', d['us_per_denoise_iteration'], 'us/iter', d.get('roofline'), d.get('cpu_baseline', {}).get('value'))"
cd /tmp && export TMPDIR=/tmp
LDM_CIN1_PK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_train -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_train.log 2>&1 \
    || { echo "rocprof failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_train.log; exit 1; }
find $GRAFT_REPO_ROOT/$OUT/prof_train -name "*stats*"
