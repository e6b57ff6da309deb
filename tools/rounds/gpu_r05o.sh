# Round 5o: batches in flight x HIP hardware queues for the 32-problem shard (--shard-of 8), where the
# kernel trace (r05n) shows the distance and bound kernels running only 32 % / 22 % of the timed region
# (the per-batch chain of latency-bound kernels limits a 12-deep pipeline); C4 at the best setting.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "host", d["host_enqueue_ms_per_step"])'; }
for cfg in "12 16" "16 16" "16 24" "20 24" "24 32" "12 16"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --shard-of 8 --inflight $1 --hw-queues $2 > $O/s8_if$1_hq$2.log 2>&1
  echo "s8 inflight $1 hwq $2: $(show $O/s8_if$1_hq$2.log)"
done
for cfg in "12 16" "16 24" "24 32"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --shard-of 4 --inflight $1 --hw-queues $2 > $O/s4_if$1_hq$2.log 2>&1
  echo "s4 inflight $1 hwq $2: $(show $O/s4_if$1_hq$2.log)"
done
for cfg in "12 16" "16 24"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --inflight $1 --hw-queues $2 > $O/c4_if$1_hq$2.log 2>&1
  echo "c4 inflight $1 hwq $2: $(show $O/c4_if$1_hq$2.log)"
done
