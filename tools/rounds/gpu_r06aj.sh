# Round 6 aj: the distance kernel's trailing-sweep pieces (MIM_KNN_TAIL=1; no effect on the full C4 batch,
# whose 5,120 sweeps fill the 512 resident blocks exactly) on the 8-GPU shard, interleaved with the
# default, three rounds -> profiles/r06aj_summary.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "knn", k.get("knn"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 > $O/base_$i.log 2>&1
  echo "base run $i: $(show $O/base_$i.log)" | tee -a $O/summary.txt
  MIM_KNN_TAIL=1 timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 > $O/tail_$i.log 2>&1
  echo "tail run $i: $(show $O/tail_$i.log)" | tee -a $O/summary.txt
done
