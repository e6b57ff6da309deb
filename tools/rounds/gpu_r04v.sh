# Round 4v: the bound kernel's tile loop software-pipelined over half tiles (next column block's MFMAs
# issued before this block's scoring) with VGPR accumulators (new) vs AGPR (pagpr), the L1 kernel
# unpipelined with VGPR (vgpr) and the previous commit (prev): bound tests, then same-box A/B on C4.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "bound or filtered or corpus" --timeout 420 --timeout-method thread > $O/pytest_bound.log 2>&1
tail -1 $O/pytest_bound.log
for v in new prev pagpr vgpr new prev pagpr vgpr; do
  if [ $v = new ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  python3 - $O/bench_c4_$v.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print('c4', sys.argv[2], d['value'], d['ms_per_step'], 'bound', d['roofline']['others']['bound']['ms_per_step'])
PY
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
