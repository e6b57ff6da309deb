# Round 5 closing tree, part 3 (after the scene configs' default of 16 hardware queues, r05v): one more
# default c1img and dataset run each (with r05v's two 16-queue runs: three per config), then the round's
# kernel traces of C4, C3, C5 and c1img (tools/prof_round.sh) -> profiles/r05_*.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R05Z_OUT:-r05z}
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("single_scene_ms"), d.get("scenes_per_s"))'; }
timeout -k 10 400 python -u bench.py --config c1img > $O/bench_c1img_3.log 2>&1; echo "c1img $(show $O/bench_c1img_3.log)"
timeout -k 10 400 python -u bench.py --config dataset > $O/bench_dataset_3.log 2>&1; echo "dataset $(show $O/bench_dataset_3.log)"
for C in c4 c3 c5 c1img; do
  timeout -k 10 900 bash tools/prof_round.sh $C
  echo "prof $C done"
done
