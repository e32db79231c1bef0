set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -k "second_step or decreases or epochs or autoencoder or train_step" --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
echo "== without the version bump:"
timeout -k 10 200 python -u -c "
import sys; sys.path[:0]=['tests','tests/golden','music-style-transfer-ldm_amd','.']
import torch; torch.autograd.graph.increment_version = lambda p: None
import conftest, test_gpu_train as T
try:
    T.test_second_step_uses_updated_weights(torch.device('cuda:0')); print('passed')
except AssertionError as e: print('FAILED', e)
" 2>&1 | tail -2
