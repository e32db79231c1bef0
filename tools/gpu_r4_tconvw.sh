#!/bin/bash
# Round 4: the window form of the 16-bit train-step conv (tconvw_kernel): parity, per-layer times against the
# per-chunk gather form (LDM_TCONV_WIN=0), the config-3 parity test and the train bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${1:-r4tcw}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled.py -x -v --timeout 240 --timeout-method thread > $O/tiled.log 2>&1
rc=$?; tail -3 $O/tiled.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tiled.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/time_conv.py bf16 > $O/time_conv_win.txt 2>&1 || { tail $O/time_conv_win.txt; exit 1; }
LDM_TCONV_WIN=0 timeout -k 10 200 python -u tools/time_conv.py bf16 > $O/time_conv_gather.txt 2>&1 || { tail $O/time_conv_gather.txt; exit 1; }
LDM_TCONV_WIN=1 timeout -k 10 200 python -u tools/time_conv.py bf16 > $O/time_conv_win1.txt 2>&1 || { tail $O/time_conv_win1.txt; exit 1; }
paste -d'\n' $O/time_conv_gather.txt $O/time_conv_win1.txt $O/time_conv_win.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_config3.py -x -q --timeout 300 --timeout-method thread > $O/config3.log 2>&1
rc=$?; tail -2 $O/config3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
python -c "import json; d=json.load(open('$O/train.json')); print('train', d['value'], d['unit'], d['ms_per_step'], 'ms')"
LDM_TCONV_WIN=0 timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_gather.json 2> $O/train_gather.err || { tail -20 $O/train_gather.err; exit 1; }
python -c "import json; d=json.load(open('$O/train_gather.json')); print('train (gather form)', d['value'], d['unit'], d['ms_per_step'], 'ms')"
LDM_TCONV_WIN=1 timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_win1.json 2> $O/train_win1.err || { tail -20 $O/train_win1.err; exit 1; }
python -c "import json; d=json.load(open('$O/train_win1.json')); print('train (window, no 4-phase)', d['value'], d['unit'], d['ms_per_step'], 'ms')"
