#!/bin/bash
# Round 6 final measurement on the final tree:   bash tools/gpu_r6_final.sh <tag>
#   1. the whole -m gpu suite and smoke();
#   2. HBM traffic per launch of the reverse loop's step kernels, fp32 and fp16 (tools/pmc_step_traffic.sh), written
#      into profiles/r06/ on the box BEFORE the bench runs (bench.py reads them for roofline.traffic);
#   3. the train step's PMC passes (tools/pmc_train.sh) -> profiles/r06/train_pmc.json;
#   4. the headline bench line + its rocprofv3 summary (tools/gpu_final.sh), the transfer / train lines + a train
#      summary (tools/gpu_workloads.sh), the stress line + its summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6final}; OUT=gpurun_out/$T; mkdir -p $OUT profiles/r06
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest -m gpu exited $rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 bash tools/pmc_step_traffic.sh $OUT/pmc_step 0 1 2 3 5 6 7 > $OUT/pmc_step.log 2>&1 || { echo "pmc_step failed"; tail $OUT/pmc_step.log; exit 1; }
DTYPE=fp16 timeout -k 10 400 bash tools/pmc_step_traffic.sh $OUT/pmc_step16 0 1 2 3 5 6 7 > $OUT/pmc_step16.log 2>&1 || { echo "pmc_step16 failed"; tail $OUT/pmc_step16.log; exit 1; }
cp $OUT/pmc_step/pmc_traffic_step.json profiles/r06/pmc_traffic_step.json
cp $OUT/pmc_step16/pmc_traffic_step.json profiles/r06/pmc_traffic_step_fp16.json
python3 -c "import json; d=json.load(open('profiles/r06/pmc_traffic_step.json')); print('fp32 bytes/launch', {k: round(v/1e6,2) for k,v in d['per_launch_bytes'].items()})"
python3 -c "import json; d=json.load(open('profiles/r06/pmc_traffic_step_fp16.json')); print('fp16 bytes/launch', {k: round(v/1e6,2) for k,v in d['per_launch_bytes'].items()})"
timeout -k 10 600 bash tools/pmc_train.sh $OUT/pmc_train > $OUT/pmc_train.log 2>&1 || { echo "pmc_train failed"; tail $OUT/pmc_train.log; exit 1; }
cp $OUT/pmc_train/summary.json profiles/r06/train_pmc.json
python3 -c "import json; d=json.load(open('profiles/r06/train_pmc.json')); print('train HBM bytes/step', d.get('step_hbm_bytes'), 'mfma util', d.get('step_mfma_util'))"
bash tools/gpu_final.sh $T/final || exit 1
bash tools/gpu_workloads.sh $T/workloads || exit 1
timeout -k 10 300 python -u bench.py --workload stress --steps 3 --warmup 1 > $OUT/stress.json 2> $OUT/stress.err \
    || { echo "stress failed"; tail -20 $OUT/stress.err; exit 1; }
cat $OUT/stress.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_stress -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload stress --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof_stress.log 2>&1 \
    || { echo "rocprof stress failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_stress.log; exit 1; }
cp $GRAFT_REPO_ROOT/profiles/r06/*.json $GRAFT_REPO_ROOT/$OUT/
echo done
