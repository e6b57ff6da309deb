# Round 4x: the per-GPU workload of each scaling point on the closing tree (diamond bound): bench.py
# --shard-of N = rank 0's shard of an N-rank C4 run, measured alone on one GPU, two runs each.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
for i in 1 2; do
  for n in 1 2 4 8; do
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of $n > $O/bench_c4_shard_of_${n}_$i.log 2>&1
    echo "shard-of $n run $i $(grep '^{"metric"' $O/bench_c4_shard_of_${n}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
