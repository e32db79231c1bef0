set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_syncbn.py tests/test_gpu_amp.py -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/host_probe.py > $O/host.log 2>&1 || { tail $O/host.log; exit 1; }
tail -1 $O/host.log
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
cut -c1-300 $O/train.json
