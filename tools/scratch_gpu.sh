set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g36; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; grep "^FAILED\|^E  " $O/gpu_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_final.sh final_r02e > gpurun_out/final_r02e.log 2>&1 || { tail -5 gpurun_out/final_r02e.log; exit 1; }
echo done
