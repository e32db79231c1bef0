#!/bin/bash
# bfold A/B: the fold parity tests, the bench-object parity, then the loop time per iteration with the fold on and
# off (tools/loop_times.py, twice around), and the headline bench line.   bash tools/gpu_r5_bfold.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bfold}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bfold.py tests/test_gpu_bench_config.py tests/test_gpu_amp.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -20; exit $rc; }
for r in 1 2; do
  for f in 1 0; do
    LDM_BNECK_FOLD=$f timeout -k 10 120 python -u tools/loop_times.py > $O/loop_${r}_$f.txt 2>&1 || { tail $O/loop_${r}_$f.txt; exit 1; }
    echo "round $r fold=$f: $(grep pairs $O/loop_${r}_$f.txt)"
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-legs --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
