#!/bin/bash
# tools/capture_wgrad_repro.py cases (mode:join:flags), each in its own process; stops at the first that does
# not exit 0 (a segfault ends the GPU work of the call).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-capwgrad}; shift; mkdir -p $O
for c in "$@"; do
  IFS=: read m j f <<< "$c"
  timeout -k 10 90 python -u tools/capture_wgrad_repro.py $m $j $f > $O/$m.$j.$f.log 2>&1
  rc=$?; echo "case $c: exit $rc :: $(tail -1 $O/$m.$j.$f.log)"
  [ $rc -eq 0 ] || exit $rc
done
