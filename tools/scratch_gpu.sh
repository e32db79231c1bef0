set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g27; mkdir -p $O
for v in "" _nt "" _nt; do
  LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$v.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench$v.json')); print('lib$v', d['value'], d['us_per_denoise_iteration'], {k: v['us'] for k, v in d['kernels'].items()})"
done
