# A/B of library variants on the distance kernel: C5 (kNN alone) and C3 isolated kNN, 2 rounds each.
# VARS="a b" -> gpurun_out/abk_<v>_<cfg>_<i>.log
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in ${VARS}; do
    for c in c5 c3; do
      MIM_LIB=$PWD/computervision_objectdetection_featurematching_amd/lib/variants/libmim_$v.so timeout -k 10 200 python3 bench.py --config $c --cpu-sample 0 --steps 10 > gpurun_out/abk_${v}_${c}_$i.log 2>&1
    done
  done
done
