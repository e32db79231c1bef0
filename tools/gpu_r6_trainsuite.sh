#!/bin/bash
# Round 6: the train-step / graph / optimizer GPU tests, then a train bench line and the sample bench's kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6train}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graph_state.py \
    tests/test_gpu_bfold.py tests/test_gpu_train.py tests/test_gpu_train_config3.py tests/test_gpu_train_fp16.py \
    tests/test_gpu_config4_rank.py tests/test_gpu_dp_graph.py tests/test_gpu_graph_streams.py \
    > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $OUT/train.json 2> $OUT/train.err \
    || { tail -20 $OUT/train.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/train.json')); print('train', round(d['ms_per_step'],4), 'ms')"
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/sample.json 2> $OUT/sample.err \
    || { tail -20 $OUT/sample.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/sample.json')); print('sample', d['value'], d['us_per_denoise_iteration'] if 'us_per_denoise_iteration' in d else '')
for k,v in d['kernels'].items(): print(k, v['us'], v['kernel'])"
