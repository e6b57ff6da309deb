# Round 4m: the check kernel fp32 checkSubset with one clarity bound per point set (collinearity and
# orientation) and fma determinants: pytest -m gpu, same-box A/B against the previous commit, kernel
# trace, sampler SQ counters.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
for v in new prev new prev; do
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "$v $(tail -1 $O/bench_c4_$v.log | cut -c1-150)"
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
K='ransac_attempt|ransac_check'
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv --kernel-include-regex "$K" \
   -d $O/pmc1 -o run -- python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/pmc1.log 2>&1


