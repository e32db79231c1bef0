#!/bin/bash
# Counter passes over the step-kernel layer timings (tools/step_times.py --no-loop --reps 5), one pass per
# counter group (rocprofv3 --pmc; FETCH_SIZE / TCC counters do not share a pass with many others).
# usage: tools/pmc_step.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmc_step}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d "$ROOT/$OUT/$2" -o p -- python3 "$ROOT/tools/step_times.py" --no-loop --reps 5 > "$ROOT/$OUT/$2.log" 2>&1 || { echo "pass $2 failed"; tail -5 "$ROOT/$OUT/$2.log"; exit 1; }; }
run "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" tcc
run "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" tcp
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" sq
