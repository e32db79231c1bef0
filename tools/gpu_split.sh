#!/bin/bash
# Sub-batch chains on separate streams: tune the B/2 shapes, then bench split 1 vs 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-split}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/tune_unet.py --shapes 8x16x64 4x16x64 --rounds 2 --dump $O/tune_table.json > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
cp music-style-transfer-ldm_amd/tuned_plans.json $O/tuned_plans.json
for sp in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --split $sp --no-cpu-baseline --no-kernel-timing > $O/bench_split$sp.json 2>> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  python -c "import json;r=json.load(open('$O/bench_split$sp.json'));print('split $sp VALUE',r['value'],'us/iter',r['us_per_denoise_iteration'])"
done
