set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g18; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_amp.py -k "wgrad" -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep "^FAILED\|^E  " $O/t.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/train$i.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/train$i.json
done
