# Round 4j: the per-GPU workload of each scaling point on one GPU (bench.py --shard-of N: rank 0's shard
# of an N-rank C4 run, 256/N problems per batch), and the host enqueue time per step at N = 8's shard
# (rocprofv3 kernel trace of the shard-of-8 line: GPU busy time vs step time).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
for n in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of $n > $O/bench_c4_shard_of_$n.log 2>&1
  echo "shard-of $n $(tail -1 $O/bench_c4_shard_of_$n.log | cut -c1-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace8 -o run -- \
  python3 bench.py --cpu-sample 0 --shard-of 8 --iso-steps 0 > $O/trace8.log 2>&1
