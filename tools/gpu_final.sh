#!/bin/bash
# Round-end style run: full bench (with CPU baseline) + rocprofv3 kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-final}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
find $O/prof -name '*stats*'
