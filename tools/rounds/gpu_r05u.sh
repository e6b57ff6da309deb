# Round 5u: the new LDS footprint defaults (3-tile distance stages, 4-tile bound chunks) against HEAD's
# (4 / 8; variants/libmim_prev.so) on C4, C3, C5 and c1img, two interleaved rounds on one box.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05u
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"], d.get("single_scene_ms"))'; }
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c5 --cpu-sample 0 --parity-sample 0 > $O/c5_${v}_$i.log 2>&1; echo "c5 $v $(show $O/c5_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_${v}_$i.log 2>&1; echo "c1img $v $(show $O/c1img_${v}_$i.log)"
  done
done
