# Round 4w: where the bound kernel's time goes — kernel traces of diagnostic builds (results invalid,
# timing only): noloop (hypotheses, staging, no tile loop), noprologue (a trivial H per lane: tile
# loop and staging only) and the committed kernel (prev).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
for v in prev noloop noprologue; do
  export MIM_LIB=$PWD/variants/libmim_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 bench.py --inflight 1 --steps 2 --warmup 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/trace_$v.log 2>&1 || true
  python3 - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bound' in r['Name'] or 'exact' in r['Name']:
        print(sys.argv[2], r['Name'][:40], r['Calls'], r['AverageNs'])
PY
done
