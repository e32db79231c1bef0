#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-actbwd}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_amp.py tests/test_gpu_train_config3.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail $O/train.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/train.json')); print('train', d['ms_per_step'], 'ms/step', d['value'], 'samples/s')"
