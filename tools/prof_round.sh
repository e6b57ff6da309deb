# Round profile for config $1 (c3 | c4 | c5 | c1img): kernel trace + stats of the isolated path
# (--inflight 1: one batch at a time, so rocprof's per-kernel averages are the launch durations the
# bench line's roofline reports), then HBM counters in separate --pmc passes.  -> gpurun_out/prof_$1/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
C=${1:-c3}
O=gpurun_out/prof_$C
rm -rf $O && mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --config $C --inflight 1 --steps 5 --warmup 1 --iso-steps 5 --cpu-sample 0 > $O/bench_trace.log 2>&1
if [ "$C" != c1img ]; then
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv \
      --kernel-include-regex 'knn2_i8|ransac_bound|ransac_attempt|ransac_check' -d $O/pmc_$P -o run -- \
      python3 bench.py --config $C --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/pmc_$P.log 2>&1
  done
  python3 tools/traffic_json.py $O $O/pmc_traffic.json $C > /dev/null
fi
