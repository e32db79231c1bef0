#!/bin/bash
# Round 3: row windows for every step layer + plane forms — parity, loop time on/off, layer times, KS sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-win2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py tests/test_gpu_attention_wide.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: step tests rc=$rc"; exit $rc; fi
for p in 11 10 00; do
  LDM_UCONV_PLANE=${p:0:1} LDM_UCONV_WINDOW=${p:1:1} timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_$p.txt 2>&1 || exit 1
  echo "plane,window $p: $(grep pairs $O/loop_$p.txt)"
done
for w in 1 0; do
  LDM_UCONV_WINDOW=$w timeout -k 10 120 python -u tools/step_times.py --no-loop --variant uconv > $O/layers_w$w.txt 2>&1 || exit 1
  echo "window $w:"; grep -v amdgpu.ids $O/layers_w$w.txt
done
MASKS="0x18 0x38 0x1c" bash tools/gpu_ks_sweep.sh $T/ks
