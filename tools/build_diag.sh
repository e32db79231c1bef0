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
# no loads, no MFMAs (-DLDM_DIAG=24): the kernel's fixed cost -> lib/libldm_amd_diag24.so
mkdir -p ../build/diag24
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DLDM_DIAG=24 -fno-gpu-rdc -x hip -c conv.hip -o ../build/diag24/conv.hip.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_diag24.so ../build/diag24/conv.hip.o ../build/diag4/capi.cpp.o ../build/diag4/misc.hip.o ../build/diag4/unet.hip.o ../build/diag4/backward.hip.o
# fixed cost with a minimal epilogue (-DLDM_DIAG=56) -> lib/libldm_amd_diag56.so
mkdir -p ../build/diag56
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DLDM_DIAG=56 -fno-gpu-rdc -x hip -c conv.hip -o ../build/diag56/conv.hip.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_diag56.so ../build/diag56/conv.hip.o ../build/diag4/capi.cpp.o ../build/diag4/misc.hip.o ../build/diag4/unet.hip.o ../build/diag4/backward.hip.o
# stamps on the fixed-cost variant (-DLDM_DIAG=60) -> lib/libldm_amd_diag60.so
mkdir -p ../build/diag60
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DLDM_DIAG=60 -fno-gpu-rdc -x hip -c conv.hip -o ../build/diag60/conv.hip.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_diag60.so ../build/diag60/conv.hip.o ../build/diag4/capi.cpp.o ../build/diag4/misc.hip.o ../build/diag4/unet.hip.o ../build/diag4/backward.hip.o
