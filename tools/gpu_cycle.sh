#!/bin/bash
# One GPU iteration: parity tests, optional autotune (TUNE=1), bench, per-block stamps.
#   bash tools/gpu_cycle.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-cycle}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
if [ "${TUNE:-0}" = 1 ]; then
  timeout -k 10 700 python -u tools/tune_unet.py --shapes 8x16x64 --rounds 2 --dump $O/tune_table.json > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
  cp music-style-transfer-ldm_amd/tuned_plans.json $O/tuned_plans.json
  grep best $O/tune.log
fi
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "
import json;r=json.load(open('$O/bench.json'));print('VALUE',r['value'],'us/iter',r['us_per_denoise_iteration'])
for k,v in r['kernels'].items(): print(f'  {k:10s} {v[\"us\"]:7.2f} us {v[\"tflops\"]:6.1f} TF', v.get('plan',''))"
if [ -f music-style-transfer-ldm_amd/lib/libldm_amd_diag4.so ] && [ "${STAMPS:-1}" = 1 ]; then
  LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd_diag4.so timeout -k 10 120 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { echo "stamp failed"; tail $O/stamps.txt; exit 1; }
  cat $O/stamps.txt
fi
