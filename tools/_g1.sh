set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step_kernels.py > gpurun_out/u5_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/step_times.py > gpurun_out/u5_base.log 2>&1 && \
LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd_ustepd4.so timeout -k 10 120 python -u tools/step_times.py --no-loop --stamps > gpurun_out/u5_d4.log 2>&1
