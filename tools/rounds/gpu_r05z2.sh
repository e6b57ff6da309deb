# Round 5 closing tree, part 2: three default runs each of c1img and dataset, and the per-GPU workload
# of the strong-scaling points (--shard-of 2, 4, 8: rank 0's shard on one GPU), two runs each
# -> profiles/r05_bench_<config>_<i>.log, r05_bench_c4_shard_of_<N>_<i>.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R05Z_OUT:-r05z}
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("single_scene_ms"), d.get("scenes_per_s"))'; }
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --config c1img > $O/bench_c1img_$i.log 2>&1; echo "c1img $(show $O/bench_c1img_$i.log)"
  timeout -k 10 400 python -u bench.py --config dataset > $O/bench_dataset_$i.log 2>&1; echo "dataset $(show $O/bench_dataset_$i.log)"
done
for i in 1 2; do
  for n in 2 4 8; do
    timeout -k 10 400 python -u bench.py --shard-of $n --cpu-sample 0 > $O/bench_c4_shard_of_${n}_$i.log 2>&1; echo "shard-of $n $(show $O/bench_c4_shard_of_${n}_$i.log)"
  done
done
