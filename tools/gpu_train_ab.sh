#!/bin/bash
# A/B of the train step (config 3, B = 32 bf16) over env settings: bench.py --workload train per setting, twice
# around, then one rocprofv3 kernel summary per setting.   bash tools/gpu_train_ab.sh <tag> <settings...>
# (a setting is space-free VAR=VALUE pairs joined by commas, as in gpu_ab.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
for rnd in 1 2; do
  i=0
  for s in "$@"; do
    i=$((i+1))
    env ${s//,/ } timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_${rnd}_$i.json 2> $O/train_${rnd}_$i.err || { tail $O/train_${rnd}_$i.err; exit 1; }
    echo "round $rnd [$s]: $(python3 -c "import json; d=json.load(open('$O/train_${rnd}_$i.json')); print(d['ms_per_step'], 'ms')")"
  done
done
i=0
for s in "$@"; do
  i=$((i+1))
  env ${s//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$i.log 2>&1 || { echo "rocprof failed"; tail $O/prof_$i.log; exit 1; }
done
