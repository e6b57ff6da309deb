# Round 3p: checkSubset decided in fp32 where it cannot disagree with fp64 (check kernel) vs the fp64
# check (variant chk64): RANSAC parity tests, isolated kernels (knn_ab), C4 and C3 lines of each.
# -> gpurun_out/r03p/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
set +e
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py tests/test_bounds_corpus_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MIM_LIB=$PWD/$V/libmim_chk64.so timeout -k 10 240 python -u tools/knn_ab.py --tag chk64 --save > $O/ab.log 2> $O/ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag chkf32 >> $O/ab.log 2>> $O/ab.err
cut -c1-420 $O/ab.log
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-150
MIM_LIB=$PWD/$V/libmim_chk64.so timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4_chk64.log 2>&1
tail -1 $O/bench_c4_chk64.log | cut -c1-150
