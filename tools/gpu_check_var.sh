# full GPU tests on the default build, then bench per variant
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
make -s -C oracle
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  MIM_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/var/$n.bench 2>&1
done
