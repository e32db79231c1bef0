#!/bin/bash
# Round 3: layer-pair launches — parity, timing, then the full -m gpu suite and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pairs}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_pairs.py -x -v --timeout 240 --timeout-method thread > $O/pair_tests.log 2>&1
rc=$?; tail -12 $O/pair_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: pair tests rc=$rc"; exit $rc; fi
timeout -k 10 240 python -u tools/pair_times.py 0 0x1 0x2 0x40 0x80 0x41 0x81 0xc2 > $O/pair_times.txt 2>&1 || { tail $O/pair_times.txt; exit 1; }
cat $O/pair_times.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: pytest -m gpu exited $rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
