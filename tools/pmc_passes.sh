#!/bin/bash
# Counter passes for one layer (separate passes: FETCH_SIZE and WRITE_SIZE do not fit together).
# usage: tools/pmc_passes.sh <layer> <outdir>
set -e
LAYER=${1:-4}; OUT=${2:-gpurun_out/pmc}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 10 120 rocprofv3 --pmc $1 -T --output-format csv -d "$ROOT/$OUT/$2" -o p -- python3 "$ROOT/tools/prof_layer.py" --layer $LAYER --reps 50 > "$ROOT/$OUT/$2.log" 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" sq1
run "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" sq2
run "FETCH_SIZE" fetch
run "WRITE_SIZE" write
