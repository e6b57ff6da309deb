# Round profile: kernel trace + stats of the default bench, then HBM counters (separate --pmc passes,
# kernel trace only) for the distance and bound kernels.  Outputs under gpurun_out/prof_round/.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_round
rm -rf $O && mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-timing > $O/bench_trace.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex 'knn2_i8|ransac_bound|ransac_attempt|ransac_check' \
     -d $O/pmc_$C -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $O/pmc_$C.log 2>&1
done
python3 tools/traffic_json.py $O $O/pmc_traffic.json > /dev/null
