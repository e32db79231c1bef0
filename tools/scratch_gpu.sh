set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; grep "^FAILED\|^E  " $O/gpu_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_workloads.sh workloads_r02d > gpurun_out/workloads_r02d.log 2>&1 || { tail -5 gpurun_out/workloads_r02d.log; exit 1; }
echo done
