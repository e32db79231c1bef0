#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-fold2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_bench_config.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/pair_times.py 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof failed"; tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
grep -h "fold_keys" $GRAFT_REPO_ROOT/$O/prof/*kernel_stats.csv | cut -c1-200
cd $GRAFT_REPO_ROOT && timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop.txt 2>&1 && echo "loop: $(grep pairs $O/loop.txt)"
for k in 1 0 1 0; do LDM_FOLD_KEYS4=$k timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_k4_$k.txt 2>&1 || exit 1; echo "keys4 $k: $(grep pairs $O/loop_k4_$k.txt)"; done
