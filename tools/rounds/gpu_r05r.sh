# Round 5r: batches on streams of mixed priority (MIM_BENCH_PRIO=k: every k-th context's stream high),
# to break the convoys in which no batch has its distance or bound kernel ready (r05n: neither runs
# 8.7 % of the C4 timed region); C4 and the 32-problem shard, two interleaved rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05r
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "host", d["host_enqueue_ms_per_step"])'; }
for i in 1 2; do
  for pr in 0 2 4 16; do
    if [ $pr = 0 ]; then unset MIM_BENCH_PRIO; else export MIM_BENCH_PRIO=$pr; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 > $O/c4_p${pr}_$i.log 2>&1; echo "c4 prio $pr: $(show $O/c4_p${pr}_$i.log)"
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 --shard-of 8 > $O/s8_p${pr}_$i.log 2>&1; echo "s8 prio $pr: $(show $O/s8_p${pr}_$i.log)"
  done
done
