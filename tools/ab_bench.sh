# A/B of library variants on the bench's isolated kernel times: VARS="a b" ARGS="--steps 10" -> gpurun_out/ab_<v>_<i>.log
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in ${VARS}; do
    MIM_LIB=$PWD/computervision_objectdetection_featurematching_amd/lib/variants/libmim_$v.so timeout -k 10 200 python3 bench.py --cpu-sample 0 ${ARGS:---steps 10} > gpurun_out/ab_${v}_$i.log 2>&1
  done
done
