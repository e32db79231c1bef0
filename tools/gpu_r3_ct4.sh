#!/bin/bash
# convT 64 -> 1 test + train bench + train kernel summary (split channel walk with prefetch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-ct4}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiled.py -k cout1 tests/test_gpu_parity.py::test_vae_and_style_encoder tests/test_gpu_train_config3.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --workload train --steps 7 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); grep -h convT4 "$f"
grep -h '"value"' $O/prof.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('train', d['ms_per_step'])"
