#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run -> gpurun_out/<tag>/prof (csv summary)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
find $O/prof -name '*stats*'
