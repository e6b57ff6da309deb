# Round 3ab: kernel trace of the N = 8 per-GPU workload (bench.py --shard-of 8), GPU busy fraction in the
# timed region.  -> gpurun_out/r03ab/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python3 bench.py --shard-of 8 --cpu-sample 0 --steps 200 --iso-steps 1 > $O/bench.log 2>&1
grep "^{" $O/bench.log | tail -1 | cut -c1-200
python3 tools/busy_frac.py $O/trace/run_kernel_trace.csv 0.45 0.85
