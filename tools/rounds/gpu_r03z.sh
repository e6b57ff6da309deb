# Round 3z: C4 per-GPU workload at N = 8 (bench.py --shard-of 8: 32 problems per batch): batches in
# flight 8 / 12 / 16 / 24 and hardware queues 16 / 24.  -> gpurun_out/r03z/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
for cfgs in "12 16" "8 16" "16 16" "24 24" "16 24" "12 16"; do
  set -- $cfgs
  timeout -k 10 400 python -u bench.py --shard-of 8 --cpu-sample 0 --steps 60 --inflight $1 --hw-queues $2 --iso-steps 2 > $O/bench_if$1_q$2.log 2>&1
  tail -1 $O/bench_if$1_q$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight $1 queues $2', d['value'], d['ms_per_step'])"
done
