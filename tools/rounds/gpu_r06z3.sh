# Round 6 closing tree, part 3: the per-GPU rate of the 8-GPU strong-scaling point against the full batch
# on the same box, interleaved, three runs each (bench.py --shard-of 8: rank 0's 32-problem shard on one
# GPU) -> profiles/r06_bench_c4_full_<i>.log, r06_bench_c4_shard_of_8_<i>.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4_full_$i.log 2>&1; echo "full $(show $O/bench_c4_full_$i.log)"
  timeout -k 10 400 python -u bench.py --shard-of 8 --cpu-sample 0 > $O/bench_c4_shard_of_8_$i.log 2>&1; echo "shard-of 8 $(show $O/bench_c4_shard_of_8_$i.log)"
done
