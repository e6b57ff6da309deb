# Round 3bc: early tiles of the distance kernel as branch-free top-2 of 32-bit (D, row) keys (3 VALU per
# value) vs the (D, index) insertion (old), and longer early phases (e8, e12): kNN parity tests, isolated
# C3/C5 A/B alternating, pipelined C4.  -> gpurun_out/r03bc/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bc
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
set +e
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit 1; fi
MIM_LIB=$V/libmim_old.so timeout -k 10 240 python -u tools/knn_ab.py --tag old --save > $O/ab.log 2> $O/ab.err
for rep in 1 2; do
  timeout -k 10 200 python -u tools/knn_ab.py --tag keys4 >> $O/ab.log 2>> $O/ab.err
  MIM_LIB=$V/libmim_e8.so timeout -k 10 200 python -u tools/knn_ab.py --tag keys8 >> $O/ab.log 2>> $O/ab.err
  MIM_LIB=$V/libmim_e12.so timeout -k 10 200 python -u tools/knn_ab.py --tag keys12 >> $O/ab.log 2>> $O/ab.err
  MIM_LIB=$V/libmim_old.so timeout -k 10 200 python -u tools/knn_ab.py --tag old >> $O/ab.log 2>> $O/ab.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03bc/ab.log"):
    d = json.loads(l); print(d["tag"], "c3 knn", d["c3_knn_ms"], "c5 knn", d["c5_knn_ms"], d["parity"][:30])
PY
for rep in 1 2; do
  for L in default e8 old; do
    if [ $L = default ]; then LIB=""; else LIB=$V/libmim_$L.so; fi
    MIM_LIB=$LIB timeout -k 10 300 python -u bench.py --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $L', d['value'], d['ms_per_step'])"
  done
done
