# Round 4t: the bound kernel with VGPR MFMA accumulators (waves_per_eu(2): no v_accvgpr_read per
# result): the bound tests, same-box A/B against the previous commit on C4 and C3, kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "bound or filtered or corpus" --timeout 420 --timeout-method thread > $O/pytest_bound.log 2>&1
tail -1 $O/pytest_bound.log
for v in new prev new prev; do
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "c4 $v $(tail -1 $O/bench_c4_$v.log | cut -c1-150)"
done
for v in new prev; do
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
  timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3_$v.log 2>&1
  echo "c3 $v $(tail -1 $O/bench_c3_$v.log | cut -c1-150)"
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
