# Round 6 w: batches in flight and hardware queues on the 8-GPU shard (bench.py --shard-of 8, 32 problems
# per step), interleaved, two rounds -> profiles/r06w_shard_inflight_ab.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2; do
  for v in "16 24" "24 32" "32 32" "12 16" "8 16"; do
    set -- $v
    timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 --inflight $1 --hw-queues $2 > $O/shard_if$1_q$2_$i.log 2>&1
    echo "inflight=$1 queues=$2 run $i: $(show $O/shard_if$1_q$2_$i.log)" | tee -a $O/summary.txt
  done
done
