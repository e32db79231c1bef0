mkdir -p gpurun_out/d1
for v in "" _uconvd1 _uconvd2 _uconvd3; do
  LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd$v.so timeout -k 10 120 python -u tools/step_times.py --no-loop --variant uconv > gpurun_out/d1/times$v.txt 2>&1 || exit 1
done
LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd_uconvd4.so timeout -k 10 120 python -u tools/step_times.py --no-loop --variant uconv --stamps > gpurun_out/d1/stamps.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/d1/bench.json 2> gpurun_out/d1/bench.err || exit 1
tail -n 12 gpurun_out/d1/*.txt
python3 -c "import json;d=json.load(open('gpurun_out/d1/bench.json'));print(d['value'],d['us_per_denoise_iteration']);[print(k,v['us'],v['kernel']) for k,v in d['kernels'].items()]"
