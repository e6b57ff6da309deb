# r06s: (1) SIFT / pipeline GPU tests on the current tree (keypoint sort: a stage's reads issued before its
# (3) kernel trace of c1img single scenes.
# exchanges); (2) c1img lines prev (HEAD sift.hip) vs cur x2;
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
CUR=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_sift_gpu.py tests/test_golden_gpu.py tests/test_pipeline_gpu.py tests/test_sift_limits_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_sift.log 2>&1 || rc=$?
tail -3 $O/pytest_sift.log
case $rc in 0) ;; *) echo "pytest rc $rc: stopping"; exit 1;; esac
for i in 1 2; do
  for v in prev cur; do
    L=$V/libmim_$v.so; [ $v = cur ] && L=$CUR
    MIM_LIB=$L timeout -k 10 300 python3 -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img_${v}_$i.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1img -o run -- \
  python3 bench.py --config c1img --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/c1img_trace_bench.log 2>&1 < /dev/null
python3 tools/scene_timeline.py $O/c1img/run_kernel_trace.csv 4 > $O/c1img_timeline.txt
echo done
