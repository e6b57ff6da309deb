# Round 3bj: distance-kernel timing probes on the closing kernel (results invalid for the probes):
# nohit = the late filter without insertion events, nosel = no selection (xor of the accumulators),
# mfmaonly = one accumulator read per column tile.  -> gpurun_out/r03bj/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bj
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
for rep in 1 2; do
  for L in nohit nosel mfmaonly; do
    MIM_LIB=$V/libmim_$L.so timeout -k 10 200 python -u tools/knn_ab.py --tag $L >> $O/ab.log 2>> $O/ab.err || true
  done
  timeout -k 10 200 python -u tools/knn_ab.py --tag default >> $O/ab.log 2>> $O/ab.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03bj/ab.log"):
    d = json.loads(l); print(d["tag"], "c3 knn", d["c3_knn_ms"], "c5 knn", d["c5_knn_ms"])
PY
