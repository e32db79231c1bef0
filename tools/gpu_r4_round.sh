#!/bin/bash
# Round 4: autocast output semantics (LDM_DT_ROUND_OUT / LDM_ACT_ROUND_*): the reduced-precision parity tests with
# their distance tables printed, with and without the output rounding (LDM_AMD_AUTOCAST_OUT=0), then the train
# and transfer bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4round}; O=$PWD/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_amp.py tests/test_gpu_train_config3.py -v -s --timeout 300 --timeout-method thread > $O/amp_round.log 2>&1
rc=$?; grep -E "PASS|FAIL|ref bf16-vs|ours vs" $O/amp_round.log | head -80; tail -2 $O/amp_round.log
LDM_AMD_AUTOCAST_OUT=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_amp.py tests/test_gpu_train_config3.py -v -s --timeout 300 --timeout-method thread -k "train or content_style or ddim10" > $O/amp_noround.log 2>&1
grep -E "PASS|FAIL|ref bf16-vs|ours vs" $O/amp_noround.log | head -60; tail -2 $O/amp_noround.log
rc0=$rc; grep -E "^E  |^FAILED" $O/amp_round.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_batched_repack.py tests/test_gpu_tiled.py tests/test_gpu_step_kernels.py -x -q --timeout 300 --timeout-method thread > $O/other.log 2>&1
rc=$?; tail -2 $O/other.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/other.log | head; exit $rc; }
timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
python -c "import json; d=json.load(open('$O/train.json')); print('train', d['value'], d['unit'], d['ms_per_step'], 'ms')"
timeout -k 10 240 python -u bench.py --workload transfer --steps 10 --warmup 2 --no-cpu-baseline > $O/transfer.json 2> $O/transfer.err || { tail -20 $O/transfer.err; exit 1; }
python -c "import json; d=json.load(open('$O/transfer.json')); print('transfer', d['value'], d['unit'], d['us_per_denoise_iteration'], 'us/iter')"
exit $rc0
