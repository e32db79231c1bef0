set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/b2.json 2> gpurun_out/b2.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/b2prof -o p -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/b2prof.json 2> $R/gpurun_out/b2prof.err
