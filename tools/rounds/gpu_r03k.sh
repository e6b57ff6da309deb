# Round 3k: register-resident Jacobi (jacobi_wave<8>) for the refine's LM solves vs the LDS group
# version (variant jgroup): RANSAC/pipeline parity tests, C3 isolated kernels (knn_ab), c1img line.
# -> gpurun_out/r03k/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
set +e
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/knn_ab.py --tag jwave --save > $O/ab.log 2> $O/ab.err
MIM_LIB=$PWD/$V/libmim_jgroup.so timeout -k 10 200 python -u tools/knn_ab.py --tag jgroup >> $O/ab.log 2>> $O/ab.err
cut -c1-420 $O/ab.log
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-200
