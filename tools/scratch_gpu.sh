set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g29; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_tiled.py -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; grep "^FAILED\|^E  " $O/t.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_conv.py bf16 > $O/conv.log 2>&1 || { tail $O/conv.log; exit 1; }
grep "enc1 k3s2 1\|dec3" $O/conv.log
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/train.json
