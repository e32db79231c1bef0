#!/bin/bash
# GPU check of the tree: every -m gpu test (no early stop), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-v}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "FAILED: pytest -m gpu exited $rc (bench not run)"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
