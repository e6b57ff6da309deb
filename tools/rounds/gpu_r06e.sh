# r06e: SIFT latency.  (1) same-address atomic probe; (2) the SIFT / pipeline GPU tests on the current tree
# (DoG planes written by the blurs, LDS-tiled extrema test with one counter atomic per block); (3) SIFT
# times and c1img lines: prev (HEAD sift.hip) / cur / orient probes (timing only); (4) kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 120 ./tools/atomic_probe > $O/atomic_probe.txt 2>&1
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_sift_gpu.py tests/test_golden_gpu.py tests/test_pipeline_gpu.py tests/test_sift_limits_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_sift.log 2>&1 || rc=$?
tail -3 $O/pytest_sift.log
case $rc in 124|134|137|139) echo "pytest rc $rc: stopping"; exit 1;; esac
for i in 1 2; do
  for v in prev cur ori1 ori2; do
    L=$V/libmim_$v.so
    [ $v = cur ] && L=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
    MIM_LIB=$L timeout -k 10 120 python3 -u tools/time_sift.py --reps 20 > $O/time_sift_${v}_$i.log 2>&1
  done
  for v in prev cur; do
    L=$V/libmim_$v.so
    [ $v = cur ] && L=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
    MIM_LIB=$L timeout -k 10 300 python3 -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img_${v}_$i.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1img -o run -- \
  python3 bench.py --config c1img --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/c1img_trace_bench.log 2>&1 < /dev/null
python3 tools/scene_timeline.py $O/c1img/run_kernel_trace.csv 4 > $O/c1img_timeline.txt
echo done
