set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g16; mkdir -p $O
for i in 1 2; do
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/train$i.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/train$i.json
done
timeout -k 10 240 python -u bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline --train-eager > $O/train_eager.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/train_eager.json
