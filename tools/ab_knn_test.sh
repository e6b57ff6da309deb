# Variants of the distance kernel: kNN parity tests, then C5 and C3 (isolated kNN) once each.
# VARS="a b" -> gpurun_out/abt_<v>.*
cd $GRAFT_REPO_ROOT
for v in ${VARS}; do
  so=$PWD/computervision_objectdetection_featurematching_amd/lib/variants/libmim_$v.so
  MIM_LIB=$so timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/abt_$v.test 2>&1
  rc=$?; echo "$v test rc=$rc $(tail -1 gpurun_out/abt_$v.test)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  for c in c5 c3; do
    MIM_LIB=$so timeout -k 10 200 python3 bench.py --config $c --cpu-sample 0 --steps 10 > gpurun_out/abt_${v}_$c.log 2>&1 || { echo "$v $c failed"; exit 1; }
  done
done
