set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g9; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_train -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_train.log 2>&1 || { echo "rocprof failed"; tail $GRAFT_REPO_ROOT/$O/prof_train.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $GRAFT_REPO_ROOT/$O/prof_train.log
