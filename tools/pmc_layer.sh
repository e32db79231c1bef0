#!/bin/bash
# Counter passes for one UNet layer kernel (separate passes).  usage: tools/pmc_layer.sh <layer> <outdir>
set -o pipefail
LAYER=${1:-9}; OUT=${2:-gpurun_out/pmc}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d "$ROOT/$OUT/$2" -o p -- python3 "$ROOT/tools/prof_layer.py" --layer $LAYER --reps 50 > "$ROOT/$OUT/$2.log" 2>&1 || { echo "pass $2 failed"; tail -5 "$ROOT/$OUT/$2.log"; exit 1; }; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" sq1
run "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" tcc
run "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TA_TCP_STATE_READ_sum" tcp
run "TA_BUSY_avr TA_TA_BUSY_sum" ta
echo done
