#!/bin/bash
# Reverse-loop time per iteration for K-split layer masks (LDM_UCONV_KS) at the default ustep layers.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ks}; mkdir -p $O
for m in ${MASKS:-0x18 0x38 0x58 0x78 0x1c 0x10 0x08 0x00}; do
  LDM_UCONV_KS=$m timeout -k 10 120 python -u tools/pair_times.py 0 > $O/loop_$m.txt 2>&1 || exit 1
  echo "ks mask $m: $(grep pairs $O/loop_$m.txt)"
done
