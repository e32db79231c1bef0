#!/bin/bash
# train-step tests + train bench + its rocprofv3 kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-wred}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_amp.py tests/test_gpu_train_config3.py tests/test_gpu_tiled.py tests/test_gpu_parity.py::test_vae_and_style_encoder -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
timeout -k 10 240 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail $O/train.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/train.json')); print('train', d['ms_per_step'], 'ms/step', d['value'], 'samples/s')"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --workload train --steps 7 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/train_kernel_stats.csv
python3 - "$O/train_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.2f}")
PY
