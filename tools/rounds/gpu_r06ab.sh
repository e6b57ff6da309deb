# Round 6 ab: kernel trace of the isolated C4 path with the deferred-check kernel
# -> profiles/r06ab_kernel_stats_c4.csv
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ab
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/bench_trace.log 2>&1
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r06ab/kernel_stats.csv")))[:16]:
    print(r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"])/1e3, 1), "us")
PY
