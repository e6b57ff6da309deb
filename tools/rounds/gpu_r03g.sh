# Round 3g: descriptor kernel with per-bin pixel masks (SIFT parity tests + c1img line); distance
# schedule A/B (MIM_KNN_SUB: legacy sweeps, segments, rounds of ~64/128/160 tiles) and the
# software-pipelined late loop (pipe*: 2 waves/SIMD), C3 HBM counters per schedule.  -> gpurun_out/r03g/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests/test_sift_gpu.py tests/test_pipeline_gpu.py tests/test_dataset_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_sift.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -3 $O/pytest_sift.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag legacy --save > $O/ab.log 2> $O/ab.err
for S in 0 64 128 160; do
  MIM_KNN_SUB=$S timeout -k 10 200 python -u tools/knn_ab.py --tag sub$S >> $O/ab.log 2>> $O/ab.err
done
for v in pipe pipes8 pipew4; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> $O/ab.log 2>> $O/ab.err
  MIM_KNN_SUB=128 MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag ${v}_sub128 >> $O/ab.log 2>> $O/ab.err
done
cut -c1-160 $O/ab.log; grep -o '"parity": "[^"]*"' $O/ab.log | cut -c1-80
for S in -1 128; do
  MIM_KNN_SUB=$S timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex knn2_i8 \
    -d $O/pmc_sub$S -o run -- python3 tools/knn_ab.py --tag pmc --c3-only --steps 2 > $O/pmc_sub$S.log 2>&1
done
echo done
