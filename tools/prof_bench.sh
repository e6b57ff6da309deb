# rocprofv3 kernel trace + stats of the default bench command itself (so the per-launch averages can
# be checked against the bench's own HIP-event times: tools/prof_window.py)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_bench
rm -rf $O && mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/bench.log 2>&1
python3 tools/prof_window.py $O/trace/run_kernel_trace.csv $O/bench.log > $O/window.json
