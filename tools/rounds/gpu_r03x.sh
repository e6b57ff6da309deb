# Round 3x: where the c1img line's time goes with 12 scenes in flight: kernel trace of the default bench,
# GPU busy fraction (tools/busy_frac.py).  -> gpurun_out/r03x/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python3 bench.py --config c1img --cpu-sample 0 --iso-steps 0 --steps 40 > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
python3 tools/busy_frac.py $O/trace/run_kernel_trace.csv 0.55 0.95
