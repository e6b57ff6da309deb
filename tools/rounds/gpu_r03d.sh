# Round 3d: the round-end checks on the current tree (pytest -m gpu as the driver runs it, smoke),
# the bench lines (c4 default, c3, c5, c1img) and the C3 profile (isolated trace + HBM counters).
# Output: gpurun_out/r03d/.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
# test failures (rc 1) do not stop the benches; a crash, abort or time limit does
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.log 2>&1
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
bash tools/prof_round.sh c3 > $O/prof_c3.log 2>&1
tail -1 $O/pytest_gpu.log
for f in c4 c3 c5 c1img; do tail -1 $O/bench_$f.log | cut -c1-300; done
# distance-kernel timing probes (results invalid): staging cost, barrier cost
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
for v in nodma nobar nosel noselnodma; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> $O/ab.log 2>> $O/ab.err
done
cat $O/ab.log
