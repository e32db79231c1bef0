#!/bin/bash
# HBM traffic per launch of the reverse loop's step kernels (rocprofv3 --pmc, one counter per pass, as
# MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE doubled for 16-B-per-lane reads, WRITE_SIZE
# as is), over tools/step_times.py --variant hybrid; summarised by tools/pmc_step_traffic.py.
#   [DTYPE=fp16] bash tools/pmc_step_traffic.sh <outdir> <layer> [<layer> ...]
set -o pipefail
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$ROOT/$OUT/l${L}_$C" -o p -- python3 "$ROOT/tools/step_times.py" --no-loop --layers $L --reps 20 --dtype ${DTYPE:-fp32} > "$ROOT/$OUT/l${L}_$C.log" 2>&1 || { echo "pass $L $C failed"; tail -5 "$ROOT/$OUT/l${L}_$C.log"; exit 1; }
  done
done
python3 "$ROOT/tools/pmc_step_traffic.py" "$ROOT/$OUT" "$@"
