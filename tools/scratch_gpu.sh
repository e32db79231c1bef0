set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g28; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -k "graphed or second_step" --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep "^FAILED\|^E  " $O/t.log | head
exit $rc
