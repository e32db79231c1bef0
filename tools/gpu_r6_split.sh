#!/bin/bash
# Round 6: the reverse loops as 1 / 2 / 4 concurrent sub-batch chains (bench.py --split; one graph per chain on its
# own stream), config 2 (fp32) and config 5 (fp16), two rounds each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6split}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for round in 1 2; do
  for sp in 1 2 4; do
    timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --split $sp --no-cpu-baseline --no-kernel-timing \
        > $OUT/sample_${sp}_${round}.json 2> $OUT/sample.err || { tail -20 $OUT/sample.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/sample_${sp}_${round}.json')); print('sample split $sp', d['us_per_denoise_iteration'], 'us/iter')"
    timeout -k 10 180 python -u bench.py --workload transfer --steps 10 --warmup 2 --split $sp --no-cpu-baseline --no-kernel-timing \
        > $OUT/transfer_${sp}_${round}.json 2> $OUT/transfer.err || { tail -20 $OUT/transfer.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/transfer_${sp}_${round}.json')); print('transfer split $sp', d['us_per_denoise_iteration'], 'us/iter')"
  done
done
