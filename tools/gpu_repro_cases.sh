#!/bin/bash
# Run a capture repro script once per case (fields of a case, ':'-separated, become its arguments), each in its
# own process; stops at the first case that does not exit 0.   bash tools/gpu_repro_cases.sh <tag> <script> case...
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:?tag}; S=${2:?script}; shift 2; mkdir -p $O
for c in "$@"; do
  timeout -k 10 90 python -u $S ${c//:/ } > $O/${c//:/.}.log 2>&1
  rc=$?; echo "case $c: exit $rc :: $(tail -1 $O/${c//:/.}.log)"
  [ $rc -eq 0 ] || exit $rc
done
