set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_amp.py -k "wgrad" -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -15 $O/t.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/time_wgrad.py bf16 > $O/time.log 2>&1 || { tail $O/time.log; exit 1; }
cat $O/time.log
