# Round 5v: the dataset line (reference's whole run, 12 scenes in flight) read 146-152k problems/s on the
# closing tree against 169k in round 4: hardware queues 24 (round 5 default) against 16.
# against round 4's closing library (variants/libmim_r04.so), dataset and c1img, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("single_scene_ms"), d.get("scenes_per_s"))'; }
for i in 1 2; do
  for v in "new 24" "new 16"; do
    set -- $v
    if [ $1 = r04 ]; then export MIM_LIB=$PWD/variants/libmim_r04.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --config dataset --cpu-sample 0 --parity-sample 0 --hw-queues $2 > $O/dataset_$1_hq$2_$i.log 2>&1; echo "dataset $1 hq $2: $(show $O/dataset_$1_hq$2_$i.log)"
    timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 --hw-queues $2 > $O/c1img_$1_hq$2_$i.log 2>&1; echo "c1img $1 hq $2: $(show $O/c1img_$1_hq$2_$i.log)"
  done
done
