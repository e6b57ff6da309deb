# Round 3h: bound kernel, x-coordinate upper bound in chunk 2 (bxonly: 3 VALU per pair) vs default;
# isolated kernels + parity (knn_ab), C3 pipelined bench line of each.  -> gpurun_out/r03h/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
MIM_LIB=$PWD/$V/libmim_bxonly.so timeout -k 10 200 python -u tools/knn_ab.py --tag bxonly >> $O/ab.log 2>> $O/ab.err
cut -c1-600 $O/ab.log
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3.log 2>&1
tail -1 $O/bench_c3.log | cut -c1-200
MIM_LIB=$PWD/$V/libmim_bxonly.so timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3_bxonly.log 2>&1
tail -1 $O/bench_c3_bxonly.log | cut -c1-200
MIM_LIB=$PWD/$V/libmim_bxonly.so timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_bounds_corpus_gpu.py tests/test_configs_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_bxonly.log 2>&1
tail -3 $O/pytest_bxonly.log
