#!/bin/bash
# HBM traffic per launch of UNet conv layers from rocprofv3 counters (separate FETCH / WRITE passes,
# MI355X_MICROARCH.md HBM section), summarised into profiles/pmc_traffic.json by tools/pmc_traffic.py.
#   bash tools/pmc_traffic.sh <outdir> <layer> [<layer> ...]
set -o pipefail
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$ROOT/$OUT/l${L}_$C" -o p -- python3 "$ROOT/tools/prof_layer.py" --layer $L --reps 50 > "$ROOT/$OUT/l${L}_$C.log" 2>&1 || { echo "pass $L $C failed"; tail -5 "$ROOT/$OUT/l${L}_$C.log"; exit 1; }
  done
done
python3 "$ROOT/tools/pmc_traffic.py" "$ROOT/$OUT" "$@"
