# r06c: single-scene latency.  (1) the GPU suite (descriptor kernel split by patch width, one-launch
# scale set copies, one-call inlier gather); (2) c1img and dataset lines x2; (3) kernel + HIP runtime
# trace of single c1img scenes (--inflight 1): tools/scene_timeline.py and the host calls in the gaps.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -3 $O/pytest_gpu.log
case $rc in 124|134|137|139) echo "pytest rc $rc: stopping"; exit 1;; esac
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img_$i.log 2>&1
  timeout -k 10 300 python3 -u bench.py --config dataset --cpu-sample 0 > $O/bench_dataset_$i.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --output-format csv -d $O/c1img -o run -- \
  python3 bench.py --config c1img --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/c1img_trace_bench.log 2>&1 < /dev/null
python3 tools/scene_timeline.py $O/c1img/run_kernel_trace.csv 4 > $O/c1img_timeline.txt
echo done
