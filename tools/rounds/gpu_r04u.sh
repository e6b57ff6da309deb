# Round 4u: the bound kernel's L1 (diamond) test in place of the box (v_sub/v_add with |.| operands
# instead of v_med3): the bound tests, then same-box A/B on C4 against the previous commit
# (variants/libmim_prev.so) and the L1 kernel with VGPR accumulators (variants/libmim_vgpr.so).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "bound or filtered or corpus" --timeout 420 --timeout-method thread > $O/pytest_bound.log 2>&1
tail -1 $O/pytest_bound.log
for v in new prev vgpr new prev vgpr; do
  if [ $v = new ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "c4 $v $(tail -1 $O/bench_c4_$v.log | cut -c1-120)"
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
