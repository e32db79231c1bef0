#!/bin/bash
# split-K kernel: GPU parity, full autotune at config-2 shape, bench with the tuned plans.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r1b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 700 python -u tools/tune_unet.py --shapes 8x16x64 --rounds 2 --dump $O/tune_table.json > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
cp music-style-transfer-ldm_amd/tuned_plans.json $O/tuned_plans.json
cat $O/tune.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
