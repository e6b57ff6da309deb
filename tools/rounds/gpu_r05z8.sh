# Round 5 closing tree (with the candidate prescreen), part 3: the round's kernel traces and HBM counters of
# C4, C3, C5 and c1img (tools/prof_round.sh) and the 2-rank launcher on the one GPU (gloo record gather).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in c4 c3 c5 c1img; do
  timeout -k 10 900 bash tools/prof_round.sh $C
  echo "prof $C done"
done
O=gpurun_out/r05z8
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 8 --cpu-sample 0 > $O/bench_c4_gloo2.log 2>&1
tail -1 $O/bench_c4_gloo2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["n_gpus"], d.get("ranks_seen"), d["gather"]["records"], d["gather"]["status_counts"], d["parity"]["checked"], d["parity"]["mismatch"])'
