set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --workload train --dtype fp32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/t8_fp32.json 2> gpurun_out/t8_fp32.err && \
timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/t8_bf16.json 2> gpurun_out/t8_bf16.err
