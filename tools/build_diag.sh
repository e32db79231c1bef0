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
# no-operand-load variant (-DLDM_DIAG=8) -> lib/libldm_amd_diag8.so (conv.hip only differs)
mkdir -p ../build/diag8
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DLDM_DIAG=8 -fno-gpu-rdc -x hip -c conv.hip -o ../build/diag8/conv.hip.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_diag8.so ../build/diag8/conv.hip.o ../build/diag4/capi.cpp.o ../build/diag4/misc.hip.o ../build/diag4/unet.hip.o ../build/diag4/backward.hip.o
