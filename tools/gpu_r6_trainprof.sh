#!/bin/bash
# Round 6: where the train step's time goes on the current tree: per-call conv timings and a rocprofv3 kernel
# summary of the graphed train bench (7 replays: 2 warm-up + 5 timed).   bash tools/gpu_r6_trainprof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-r6trainprof}
mkdir -p $O
export PYTHONUNBUFFERED=1
true
true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1 || { echo "rocprof failed"; tail $O/prof_train.log; exit 1; }
find $O/prof_train -name "*stats*"
