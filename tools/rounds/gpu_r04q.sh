# Round 4q: batches in flight at the small per-GPU shards of the 4- and 8-GPU C4 lines (bench.py
# --shard-of N --inflight F, 16 hardware queues): does the default 12 hold at 32 / 64 problems per batch?
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
for rep in 1 2; do
  for f in 8 12 16; do
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 --inflight $f > $O/s8_if${f}_$rep.log 2>&1
    echo "shard8 if$f $(tail -1 $O/s8_if${f}_$rep.log | cut -c95-150)"
  done
done
for f in 8 12 16; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 4 --inflight $f > $O/s4_if${f}.log 2>&1
  echo "shard4 if$f $(tail -1 $O/s4_if${f}.log | cut -c95-150)"
done
