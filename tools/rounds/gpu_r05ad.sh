# Round 5ad: the first RANSAC chunk's length on C4 (MIM_FIRST_CHUNK: 4,096 iterations by default; chunk 1
# carries the lower bound at 7 VALU per pair, chunk 2 the upper bound alone at 4, and chunk 2's candidate
# bar is chunk 1's best): 1,024 / 2,048 / 4,096 / 8,192, isolated bound + exact time and the line, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ad
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "score", r["score"], "exact", r["exact"], "cand", r["cand"])'; }
for i in 1 2; do
  for fc in 4096 2048 1024 8192; do
    MIM_FIRST_CHUNK=$fc timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 2 --iso-steps 2 > $O/c4_fc${fc}_$i.log 2>&1; echo "first chunk $fc: $(show $O/c4_fc${fc}_$i.log)"
  done
done
