#!/bin/bash
# Round 6, batch 18 (measurement only): the stress line's kernel summary with LDM_FLASH_KH=1 (one key group per block:
# CA1's split launches then double-buffer their K / V), against the default's in profiles/r06.   bash tools/gpu_r6_batch18.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b18}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
LDM_FLASH_KH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress_kh1 -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress_kh1.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress_kh1.log; exit 1; }
echo done
