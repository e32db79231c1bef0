set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g31; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -k "train_ldm or train_autoencoder_entry" --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep "^FAILED\|^E  \|Error" $O/t.log | head -20
exit $rc
