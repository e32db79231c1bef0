set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiled.py > gpurun_out/h1_tiled.log 2>&1 ; \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amp.py tests/test_gpu_features.py tests/test_gpu_train.py > gpurun_out/h1_tests.log 2>&1 ; \
timeout -k 10 300 python -u tools/time_vggish.py > gpurun_out/h1_vgg.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/h1_train.json 2> gpurun_out/h1_train.err
