# Round 5ab: the driver times a short window (20 steps in round 4): 12 vs 16 batches in flight (24 queues)
# at --steps 20 --warmup 5, three interleaved rounds on one box.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ab
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["batches_in_flight"])'; }
for i in 1 2 3; do
  for nf in 12 16; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --parity-sample 0 --iso-steps 1 --inflight $nf > $O/c4_k20_if${nf}_$i.log 2>&1; echo "k20 inflight $nf: $(show $O/c4_k20_if${nf}_$i.log)"
  done
done
