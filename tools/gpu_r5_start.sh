#!/bin/bash
# Round-5 first box call: -m gpu suite, the headline bench (no CPU legs), and bench.py --gpus 2 on a 1-GPU box
# (must exit non-zero with the device-count message).   bash tools/gpu_r5_start.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-r5start}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-legs > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench2.out 2> $O/bench2.err
echo "bench --gpus 2 exit $?: $(tail -1 $O/bench2.err)"
