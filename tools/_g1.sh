set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_syncbn.py tests/test_gpu_amp.py > gpurun_out/f1_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/f1_train.json 2> gpurun_out/f1_train.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/f1prof -o p -- python3 $R/bench.py --workload train --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/f1prof.json 2> $R/gpurun_out/f1prof.err
