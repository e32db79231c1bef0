#!/bin/bash
# Debug run: the RCCL-captured DP train-step test alone, output uncaptured (-s), then with async error handling off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dbgdp}; mkdir -p $O
export NCCL_DEBUG=WARN TORCH_CPP_LOG_LEVEL=INFO TORCH_DISTRIBUTED_DEBUG=DETAIL
for i in 1 2; do
timeout -k 10 200 python -u -m pytest tests/test_gpu_dp_graph.py -x -v -s --timeout 150 --timeout-method thread > $O/alone_s$i.log 2>&1
echo "alone -s run $i rc=$?"
done
TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_ENABLE_MONITORING=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_dp_graph.py -x -v -s --timeout 150 --timeout-method thread > $O/alone_noaeh.log 2>&1
echo "alone noaeh rc=$?"
