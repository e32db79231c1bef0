#!/bin/bash
# Round 6 end, part B: the headline bench + its rocprofv3 summary, the secondary lines (transfer, train + its kernel
# summary, stress), the train-step PMC passes and the step kernels' HBM traffic.   bash tools/gpu_r6_endB.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6end}; O=$PWD/gpurun_out/$T; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu_final.sh $T/final || exit 1
bash tools/gpu_workloads.sh $T/workloads || exit 1
timeout -k 10 300 python -u bench.py --workload stress --steps 3 --warmup 1 > $O/stress.json 2> $O/stress.err \
    || { echo "stress failed"; tail -20 $O/stress.err; exit 1; }
cat $O/stress.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $O/prof_stress.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/pmc_train.sh gpurun_out/$T/pmc_train > $O/pmc_train.log 2>&1 || { echo "pmc_train failed"; tail $O/pmc_train.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/pmc_train/summary.json')); print('train HBM bytes/step', d.get('step_hbm_bytes'), 'mfma util', d.get('step_mfma_util'))"
timeout -k 10 400 bash tools/pmc_step_traffic.sh gpurun_out/$T/pmc_step 0 1 2 3 5 6 7 > $O/pmc_step.log 2>&1 || { echo "pmc_step failed"; tail $O/pmc_step.log; exit 1; }
tail -12 $O/pmc_step.log
