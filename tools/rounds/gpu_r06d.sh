# r06d: SIFT descriptor latency.  (1) the GPU suite on the current tree (descriptor batches prefetched:
# the next batch's patch positions and gradient loads issued before this batch's sort); (2) c1img lines,
# two interleaved rounds: pf0 (no prefetch, as round 5) / cur (prefetch) / pf1o5 (prefetch, registers
# capped for 5 blocks per CU); (3) dataset line of cur; (4) kernel trace of single c1img scenes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -3 $O/pytest_gpu.log
case $rc in 124|134|137|139) echo "pytest rc $rc: stopping"; exit 1;; esac
for i in 1 2; do
  for v in pf0 cur pf1o5; do
    L=$V/libmim_$v.so
    [ $v = cur ] && L=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
    MIM_LIB=$L timeout -k 10 300 python3 -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img_${v}_$i.log 2>&1
  done
done
timeout -k 10 300 python3 -u bench.py --config dataset --cpu-sample 0 > $O/bench_dataset_cur.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1img -o run -- \
  python3 bench.py --config c1img --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/c1img_trace_bench.log 2>&1 < /dev/null
python3 tools/scene_timeline.py $O/c1img/run_kernel_trace.csv 4 > $O/c1img_timeline.txt
echo done
