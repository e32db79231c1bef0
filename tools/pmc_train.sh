#!/bin/bash
# Config 3 counters: rocprofv3 --pmc passes over the train-step bench (B=32, bf16 autocast), one pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass), then tools/pmc_train_summary.py.
# usage: tools/pmc_train.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmc_train}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d "$ROOT/$OUT/$2" -o p -- \
    python3 "$ROOT/bench.py" --workload train --steps 2 --warmup 1 --no-cpu-baseline --train-eager > "$ROOT/$OUT/$2.log" 2>&1 \
    || { echo "pass $2 failed"; tail -5 "$ROOT/$OUT/$2.log"; exit 1; }
}
run "FETCH_SIZE" fetch
run "WRITE_SIZE" write
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" mfma
python3 "$ROOT/tools/pmc_train_summary.py" "$ROOT/$OUT" > "$ROOT/$OUT/summary.json"
