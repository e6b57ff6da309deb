# Round 5n: kernel traces of the pipelined (12 in flight) 32-problem shard (--shard-of 8) and full C4 runs,
# to compare per-problem kernel time and GPU busy fraction (tools/trace_busy.py).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/s8 -o run -- \
  python3 bench.py --cpu-sample 0 --parity-sample 0 --shard-of 8 --steps 80 --warmup 1 --iso-steps 1 > $O/s8.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c4 -o run -- \
  python3 bench.py --cpu-sample 0 --parity-sample 0 --steps 10 --warmup 1 --iso-steps 1 > $O/c4.log 2>&1
python3 tools/trace_busy.py $O/s8/run_kernel_trace.csv 0.3 > $O/s8_busy.txt || true
python3 tools/trace_busy.py $O/c4/run_kernel_trace.csv 0.3 > $O/c4_busy.txt || true
cat $O/s8_busy.txt $O/c4_busy.txt
python3 tools/trace_busy.py $O/s8/run_kernel_trace.csv --timed 12 80 > $O/s8_timed.txt
python3 tools/trace_busy.py $O/c4/run_kernel_trace.csv --timed 12 10 > $O/c4_timed.txt
