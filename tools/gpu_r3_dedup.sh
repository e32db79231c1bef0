#!/bin/bash
# Round 3: transposed-layer activation dedup — parity of the step kernels, per-layer times, loop time per
# ustep layer mask; then the full round check (tests, smoke, bench + rocprof, workloads).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-dedup}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: step tests rc=$rc"; exit $rc; fi
timeout -k 10 120 python -u tools/step_times.py --no-loop --variant uconv > $O/layers_uconv.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/step_times.py --no-loop --variant ustep --layers 0,5,7 > $O/layers_ustep.txt 2>&1 || exit 1
cat $O/layers_uconv.txt $O/layers_ustep.txt | grep -v amdgpu.ids
for m in 0xa1 0x01 0x21 0x81; do
  LDM_USTEP_LAYERS=$m timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_$m.txt 2>&1 || exit 1
  echo "ustep mask $m: $(grep pairs $O/loop_$m.txt)"
done
bash tools/gpu_round.sh $T/round
