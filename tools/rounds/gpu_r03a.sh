# Round 3: distance-kernel parity + A/B (legacy 32x32 kernel as the bit reference, then the 16x16
# deferred-epilogue variants).  Output: gpurun_out/r03a_*.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_test.log 2>&1
MIM_LIB=$PWD/$V/libmim_legacy.so timeout -k 10 240 python -u tools/knn_ab.py --tag legacy --save > gpurun_out/r03a_ab.log 2> gpurun_out/r03a_ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag ct4 >> gpurun_out/r03a_ab.log 2>> gpurun_out/r03a_ab.err
for v in ct2 ct8 ct8s8; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> gpurun_out/r03a_ab.log 2>> gpurun_out/r03a_ab.err
done
cat gpurun_out/r03a_ab.log
