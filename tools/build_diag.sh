#!/bin/bash
# Diagnostic build (per-block timestamps, -DLDM_DIAG=4) -> lib/libldm_amd_diag4.so, for tools/stamp_probe.py
set -e
cd "$(dirname "$0")/../music-style-transfer-ldm_amd/csrc"
mkdir -p ../build/diag4
for f in capi.cpp conv.hip misc.hip unet.hip backward.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DLDM_DIAG=4 -fno-gpu-rdc -x hip -c $f -o ../build/diag4/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_diag4.so ../build/diag4/*.o
