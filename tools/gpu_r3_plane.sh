#!/bin/bash
# Round 3: bottleneck 2x8-plane tap sharing — step-kernel parity, loop time with it on/off, K-split sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-plane}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_kernels.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: step tests rc=$rc"; exit $rc; fi
for p in 11 10 01 00; do
  LDM_UCONV_PLANE=${p:0:1} LDM_UCONV_WINDOW=${p:1:1} timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_plane$p.txt 2>&1 || exit 1
  echo "plane,window $p: $(grep pairs $O/loop_plane$p.txt)"
done
LDM_USTEP_LAYERS=0 timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_ustep0.txt 2>&1 || exit 1
echo "plane,window 11, enc1 on uconv: $(grep pairs $O/loop_ustep0.txt)"
LDM_UCONV_PLANE=1 timeout -k 10 120 python -u tools/step_times.py --no-loop --variant uconv > $O/layers_uconv.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/layers_uconv.txt
MASKS="0x38 0x58 0x78 0x1c 0x10" bash tools/gpu_ks_sweep.sh $T/ks
