# Round 3ac: distance work pulled dynamically from per-XCD lists (MIM_KNN_DYN=1: whole sweeps, a block
# that starts late takes less) vs the static balanced schedule: parity tests, C3 isolated kNN, pipelined
# C4 / C3 / N=8-shard lines, alternating.  -> gpurun_out/r03ac/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_knn_gpu.py tests/test_golden_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 240 python -u tools/knn_ab.py --tag static --save > $O/ab.log 2> $O/ab.err
MIM_KNN_DYN=1 timeout -k 10 200 python -u tools/knn_ab.py --tag dyn >> $O/ab.log 2>> $O/ab.err
python3 - <<'PY'
import json
for l in open("gpurun_out/r03ac/ab.log"):
    d = json.loads(l); print(d["tag"], "c3 knn", d["c3_knn_ms"], "c5 knn", d["c5_knn_ms"], d["parity"][:30])
PY
for rep in 1 2; do
  for dyn in 0 1; do
    MIM_KNN_DYN=$dyn timeout -k 10 400 python -u bench.py --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 dyn=$dyn', d['value'], d['ms_per_step'])"
    MIM_KNN_DYN=$dyn timeout -k 10 400 python -u bench.py --config c3 --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 dyn=$dyn', d['value'], d['ms_per_step'])"
    MIM_KNN_DYN=$dyn timeout -k 10 400 python -u bench.py --shard-of 8 --steps 60 --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard8 dyn=$dyn', d['value'], d['ms_per_step'])"
  done
done
