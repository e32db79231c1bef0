#!/bin/bash
# Diagnostic builds of tconv.hip (never shipped): TCONV_DIAG 1 = no gather loads, 2 = no MFMAs, 3 = neither
# -> lib/libldm_amd_tcd{1,2,3}.so, the other objects from the regular build (run `make` first).
set -e
cd "$(dirname "$0")/../music-style-transfer-ldm_amd/csrc"
OBJS=$(ls ../build/*.o | grep -v tconv.hip.o)
for d in 1 2 3; do
  mkdir -p ../build/tcd$d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DTCONV_DIAG=$d -fno-gpu-rdc \
      -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 -x hip -c tconv.hip -o ../build/tcd$d/tconv.hip.o &
done
wait
for d in 1 2 3; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_tcd$d.so $OBJS ../build/tcd$d/tconv.hip.o
done
