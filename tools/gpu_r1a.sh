#!/bin/bash
# GPU session: parity tests, bench, per-block stamp timeline, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r1a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --split 2 --no-cpu-baseline --no-kernel-timing > $O/bench_split2.json 2>&1 || exit 1
cat $O/bench_split2.json
LDM_AMD_LIB=$PWD/music-style-transfer-ldm_amd/lib/libldm_amd_diag4.so timeout -k 10 120 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { echo "stamp failed"; tail $O/stamps.txt; exit 1; }
cat $O/stamps.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof failed"; tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name '*stats*'
