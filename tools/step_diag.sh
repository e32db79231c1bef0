#!/bin/bash
# Diagnostic variants of the step kernels (csrc/uconv.hip, -DUCONV_DIAG=k) -> lib/libldm_amd_ucd<k>.so:
#   1 no MFMAs, 2 no operand loads, 3 neither (fixed cost), 4 per-block timestamps (tools/step_times.py --stamps)
set -e
cd "$(dirname "$0")/../music-style-transfer-ldm_amd/csrc"
for k in "$@"; do
  mkdir -p ../build/ucd$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DUCONV_DIAG=$k -fno-gpu-rdc -x hip -c uconv.hip -o ../build/ucd$k/uconv.hip.o &
done
wait
for k in "$@"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_ucd$k.so ../build/ucd$k/uconv.hip.o \
    ../build/capi.cpp.o ../build/conv.hip.o ../build/misc.hip.o ../build/unet.hip.o ../build/backward.hip.o ../build/reduce.hip.o
done
