#!/bin/bash
# Diagnostic variants of the step kernels -> lib/libldm_amd_<file><k>.so (never shipped; delete after use):
#   tools/step_diag.sh uconv k...   with k: 1 no MFMAs, 2 no operand loads, 3 neither (fixed cost),
#   4 per-block timestamps (tools/step_times.py --stamps)
set -e
cd "$(dirname "$0")/../music-style-transfer-ldm_amd/csrc"
f=$1; shift
D=$(echo $f | tr a-z A-Z)_DIAG
for k in "$@"; do
  mkdir -p ../build/${f}d$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -D$D=$k -fno-gpu-rdc -x hip -c $f.hip -o ../build/${f}d$k/$f.hip.o &
done
wait
others=""
for s in $(sed -n 's/^SRCS := //p' Makefile); do
  [ "$s" = "$f.hip" ] || others="$others ../build/$s.o"
done
for k in "$@"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o ../lib/libldm_amd_${f}d$k.so ../build/${f}d$k/$f.hip.o $others
done
