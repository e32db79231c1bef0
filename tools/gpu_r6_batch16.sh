#!/bin/bash
# Round 6, batch 16: the token-major flash merge (fused engine at a [1,32,16,512] latent, CA2 over 2 key splits) and
# the width-general attention suite.   bash tools/gpu_r6_batch16.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6b16}; OUT=gpurun_out/$T; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention_wide.py tests/test_gpu_shape_s.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error|assert" $OUT/tests.log | head -20; echo "tests exited $rc: stopping"; exit $rc; fi
echo done
