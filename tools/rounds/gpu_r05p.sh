# Round 5p: finer sweep of batches in flight x hardware queues around r05o's best (16 in flight, 24
# queues) on the 32-problem shard, two interleaved rounds; then C4 and C3 at the candidates.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "host", d["host_enqueue_ms_per_step"])'; }
for i in 1 2; do
for cfg in "12 16" "12 24" "14 24" "16 24" "16 20" "18 24" "16 28" "20 28"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --shard-of 8 --inflight $1 --hw-queues $2 > $O/s8_if$1_hq$2_$i.log 2>&1
  echo "s8 inflight $1 hwq $2: $(show $O/s8_if$1_hq$2_$i.log)"
done
done
for i in 1 2; do
for cfg in "12 16" "16 24" "14 24"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --inflight $1 --hw-queues $2 > $O/c4_if$1_hq$2_$i.log 2>&1
  echo "c4 inflight $1 hwq $2: $(show $O/c4_if$1_hq$2_$i.log)"
  timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 --iso-steps 1 --inflight $1 --hw-queues $2 > $O/c3_if$1_hq$2_$i.log 2>&1
  echo "c3 inflight $1 hwq $2: $(show $O/c3_if$1_hq$2_$i.log)"
done
done
