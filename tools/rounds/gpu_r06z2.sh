# Round 6 closing tree, part 2: three default runs each of C3, C5, c1img and dataset
# -> profiles/r06_bench_<config>_<i>.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("single_scene_ms"), d.get("scenes_per_s"))'; }
for i in 1 2 3; do
  for C in c3 c5 c1img dataset; do
    timeout -k 10 400 python -u bench.py --config $C > $O/bench_${C}_$i.log 2>&1; echo "$C $(show $O/bench_${C}_$i.log)"
  done
done
