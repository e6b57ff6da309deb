# Round 3aa: 12 in flight / 16 queues vs 16 / 24 at each C4 strong-scaling point's per-GPU workload
# (bench.py --shard-of N), alternating.  -> gpurun_out/r03aa/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
for n in 8 4 2 1; do
  for cfgs in "12 16" "16 24" "12 16" "16 24"; do
    set -- $cfgs
    timeout -k 10 400 python -u bench.py --shard-of $n --cpu-sample 0 --steps 60 --inflight $1 --hw-queues $2 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard-of $n inflight $1 queues $2', d['value'], d['ms_per_step'])"
  done
done
