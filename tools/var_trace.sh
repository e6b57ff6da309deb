set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${VARS:-nogather nosubset}; do
  rm -rf gpurun_out/vt_$v
  MIM_LIB=$PWD/computervision_objectdetection_featurematching_amd/lib/variants/libmim_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vt_$v -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing --inflight 1 > gpurun_out/vt_$v.log 2>&1
done
