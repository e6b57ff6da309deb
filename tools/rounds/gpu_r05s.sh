# Round 5s: how much the distance kernel's per-stage barrier costs: LDS stages of 2 and 3 tiles (one
# barrier per stage; MIM_KNN_STAGE, variants/libmim_st<k>.so) against the default 4, isolated launch
# times on C4 and C3, two interleaved rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"])'; }
for i in 1 2; do
  for v in st4 st2 st3; do
    if [ $v = st4 ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
  done
done
