set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g37; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; grep "^FAILED\|^E  " $O/t.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench$i.json')); print(d['value'], d['us_per_denoise_iteration'], {k: v['us'] for k, v in d['kernels'].items() if 'attn' in k})"
done
