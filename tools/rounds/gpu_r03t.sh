# Round 3t: batches in flight for C4 (256 problems per batch): 4 / 6 / 8 / 12 (default) / 16.
# -> gpurun_out/r03t/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
for n in 12 4 6 8 16 12; do
  timeout -k 10 400 python -u bench.py --inflight $n --cpu-sample 0 --parity-sample 0 > $O/bench_c4_if$n.log 2>&1
  tail -1 $O/bench_c4_if$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight $n', d['value'], d['ms_per_step'])"
done
