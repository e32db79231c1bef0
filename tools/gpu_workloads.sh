#!/bin/bash
# Secondary bench lines: config 5 (transfer loop) and configs 3/4 (train step), plus a rocprofv3
# kernel summary of the train step.   bash tools/gpu_workloads.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-workloads}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u bench.py --workload transfer --steps 10 --warmup 2 > $O/transfer.json 2> $O/transfer.err || { echo "transfer failed"; tail -20 $O/transfer.err; exit 1; }
cat $O/transfer.json
timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 > $O/train.json 2> $O/train.err || { echo "train failed"; tail -20 $O/train.err; exit 1; }
cat $O/train.json
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1 || { echo "rocprof failed"; tail $O/prof_train.log; exit 1; }
  find $O/prof_train -name '*stats*'
fi
