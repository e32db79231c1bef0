#!/bin/bash
# dec1 thin A/B (parity with it forced on, loop times), then the config-3 PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-last}; O=gpurun_out/$T; mkdir -p $O
LDM_UCONV_DEC1_THIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests_dec1.log 2>&1
rc=$?; tail -2 $O/tests_dec1.log
if [ $rc -ne 0 ]; then echo "FAILED: dec1-thin tests rc=$rc"; exit $rc; fi
for e in 1 0; do
  LDM_UCONV_DEC1_THIN=$e timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_dec1thin$e.txt 2>&1 || exit 1
  echo "dec1 thin $e: $(grep pairs $O/loop_dec1thin$e.txt)"
done
bash tools/pmc_train.sh gpurun_out/$T/pmc_train > $O/pmc_train.log 2>&1 || { echo "pmc_train failed"; tail $O/pmc_train.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$T/pmc_train/summary.json')); print('step hbm GB', d.get('step_hbm_bytes',0)/1e9, 'mfma util', d.get('step_mfma_util'))"
