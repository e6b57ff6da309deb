# Round 3e: SIFT on per-scale streams (parity tests + the c1img line), the round's profiles (isolated
# traces + HBM counters of C3 / C4 / C5, the c1img trace), distance-kernel probes.  -> gpurun_out/r03e/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests/test_sift_gpu.py tests/test_pipeline_gpu.py tests/test_dataset_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_sift.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/pytest_sift.log; exit $rc; fi
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
for C in c3 c5 c4; do bash tools/prof_round.sh $C > $O/prof_$C.log 2>&1; done
bash tools/prof_round.sh c1img > $O/prof_c1img.log 2>&1
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
for v in prio nodma nobar nosel noselnodma; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> $O/ab.log 2>> $O/ab.err
done
tail -2 $O/pytest_sift.log
tail -1 $O/bench_c1img.log | cut -c1-400
cat $O/ab.log | cut -c1-200
