# Round 5y: where the SIFT descriptor kernel's ~1 ms per c1img scene goes (one launch over the five
# scales, ~19.6k keypoints): timing probes with a float exp (MIM_PROBE_DESCR=1) and with phase A alone
# (=2; both wrong descriptors by design) and a 4x larger grid (MIM_DESCR_GRID=16384), rocprofv3 kernel
# stats of a short c1img run each.  Second pass (r05y2): one descriptor launch per image (MIM_DESCR_SPLIT=1), also with phase A alone.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R05Y_OUT:-r05y}
mkdir -p $O
for v in base dsplit pd2split; do
  if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
    python3 bench.py --config c1img --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 --parity-sample 0 --inflight 1 > $O/$v.log 2>&1 || true
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'descr_kernel' in r['Name'] or 'extrema' in r['Name'] or 'kp_post' in r['Name'] or 'orient' in r['Name']: print('$v', r['Name'].split('(')[0][-20:], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
