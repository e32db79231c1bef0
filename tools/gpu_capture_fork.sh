#!/bin/bash
# Side-stream fork / join cases of tools/capture_fork_repro.py, each in its own process, least likely to fail
# first; the call stops at the first case that does not exit 0 (a segfault ends the GPU work of the call).
#   bash tools/gpu_capture_fork.sh <tag> [case ...]     case = <main|worker>:<thread_local|global>:<1|0>
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-capfork}; shift; mkdir -p $O
CASES=${@:-main:thread_local:1 main:global:1 worker:global:1 worker:thread_local:1 main:thread_local:0}
for c in $CASES; do
  IFS=: read w m j <<< "$c"
  timeout -k 10 90 python -u tools/capture_fork_repro.py $w $m $j > $O/$w.$m.$j.log 2>&1
  rc=$?; echo "case $c: exit $rc :: $(tail -1 $O/$w.$m.$j.log)"
  [ $rc -eq 0 ] || exit $rc
done
