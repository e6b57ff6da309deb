# Round 3bk: prep kernel with the row norms reduced from the fragment pass (each row read once) and the
# distance kernel's events over two row groups (g 0-7, 8-15) vs HEAD (old): pytest -m gpu, isolated
# C3/C5 distance kernel, pipelined C4 alternating, kernel trace of C4 (prep time).
# -> gpurun_out/r03bk/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bk
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
set +e
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit 1; fi
MIM_LIB=$V/libmim_old.so timeout -k 10 240 python -u tools/knn_ab.py --tag old --save > $O/ab.log 2> $O/ab.err
for rep in 1 2; do
  timeout -k 10 200 python -u tools/knn_ab.py --tag groups >> $O/ab.log 2>> $O/ab.err
  MIM_LIB=$V/libmim_old.so timeout -k 10 200 python -u tools/knn_ab.py --tag old >> $O/ab.log 2>> $O/ab.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03bk/ab.log"):
    d = json.loads(l); print(d["tag"], "c3 knn", d["c3_knn_ms"], "c5 knn", d["c5_knn_ms"], d["parity"][:30])
PY
for rep in 1 2; do
  for L in default old; do
    if [ $L = default ]; then LIB=""; else LIB=$V/libmim_$L.so; fi
    MIM_LIB=$LIB timeout -k 10 300 python -u bench.py --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $L', d['value'], d['ms_per_step'])"
  done
done
for L in default old; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/$V/libmim_$L.so; fi
  MIM_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$L -o run --output-format csv -- \
    python3 bench.py --inflight 1 --steps 3 --warmup 1 --iso-steps 1 --cpu-sample 0 > $O/tr_$L.log 2>&1
  python3 - $O/tr_$L/run_kernel_stats.csv $L <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "prep_batch" in r["Name"] or "knn2_i8" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0], r["Calls"], "avg ms", round(float(r["AverageNs"]) / 1e6, 4))
PY
done
