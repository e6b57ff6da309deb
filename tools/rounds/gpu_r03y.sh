# Round 3y: the per-GPU workload of C4's strong-scaling points on one GPU (bench.py --shard-of N: rank
# 0's shard of an N-rank run), plus a 2-rank gloo rehearsal of the real launcher on the one GPU.
# -> gpurun_out/r03y/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
for n in 1 2 4 8; do
  timeout -k 10 400 python -u bench.py --shard-of $n --cpu-sample 0 --steps 40 > $O/bench_shard$n.log 2>&1
  tail -1 $O/bench_shard$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard-of $n', d['value'], d['ms_per_step'], d['config']['problems_per_gpu'])"
done
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --cpu-sample 0 --steps 10 > $O/bench_gloo2.log 2>&1
tail -1 $O/bench_gloo2.log | cut -c1-250
