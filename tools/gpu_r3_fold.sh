#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-fold}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_bench_config.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "FAILED: tests rc=$rc"; exit $rc; fi
for k in 1 0 1 0; do LDM_FOLD_KEYS8=$k timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop$k.txt 2>&1 || exit 1; echo "keys8 $k: $(grep pairs $O/loop$k.txt)"; done

