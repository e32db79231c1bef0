set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step_kernels.py > gpurun_out/u8_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/step_times.py --loop-only 1,2 > gpurun_out/u8_loop.log 2>&1
