# parity subset + bench for each lib/variants/libmim_*.so (MIM_LIB), then the default build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
make -s -C oracle
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  case $n in *nosel*) ;; *) MIM_LIB=$PWD/$so timeout -k 10 300 python -m pytest tests/test_knn_gpu.py -x -q > gpurun_out/var/$n.test 2>&1 ;; esac
  MIM_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/var/$n.bench 2>&1
done
