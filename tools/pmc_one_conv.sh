#!/bin/bash
# PMC passes over one train conv call's kernel (tools/one_conv.py), one rocprofv3 run per counter group.
#   bash tools/pmc_one_conv.sh <tag> <kernel regex> <one_conv.py args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; RX=$2; shift 2
O=$PWD/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 python3 tools/one_conv.py "$@" > $O/time.txt 2>&1 || { tail $O/time.txt; exit 1; }
cat $O/time.txt | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $O/p$i -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/one_conv.py "$@" --reps 5 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[(r["Kernel_Name"][:60], r["Counter_Name"])] += float(r["Counter_Value"])
        n[(r["Kernel_Name"][:60], r["Counter_Name"])] += 1
for (k, c), v in sorted(tot.items()):
    print(f"{k:60s} {c:28s} {v / max(1, n[(k, c)]):14.1f} per dispatch")
PY
