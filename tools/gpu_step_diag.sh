set -e
L=music-style-transfer-ldm_amd/lib
timeout -k 10 120 python -u tools/step_times.py --no-loop > gpurun_out/d0.log 2>&1
for k in 1 2 3; do LDM_AMD_LIB=$PWD/$L/libldm_amd_ucd$k.so timeout -k 10 120 python -u tools/step_times.py --no-loop > gpurun_out/d$k.log 2>&1; done
LDM_AMD_LIB=$PWD/$L/libldm_amd_ucd4.so timeout -k 10 120 python -u tools/step_times.py --no-loop --stamps > gpurun_out/d4.log 2>&1
