# Round 4i: chunk-1 lower bound from the square inscribed in the inner disc (shares the box test's
# max(|ex|, |ey|): 7 VALU per pair instead of the octagon's 10).  pytest -m gpu (bracket, filtered ==
# exact, real-data tests), chunk-1 candidate counts, same-box A/B against the previous commit (prev),
# kernel trace.  (A distance kernel without the 2nd neighbour's index in the batch path failed the
# dataset test here: a tie between one lane half's 2nd and the other's 1st needs that index.)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
lib() { case $1 in new) unset MIM_LIB;; *) export MIM_LIB=$PWD/variants/libmim_$1.so;; esac; }
for v in new prev; do
  lib $v
  MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c4 --steps 1 --warmup 0 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand_c4_$v.log 2>&1
  MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c1img --steps 1 --warmup 0 --inflight 1 --iso-steps 1 --cpu-sample 0 > $O/ncand_c1img_$v.log 2>&1
done
for v in new prev new prev; do
  lib $v
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "$v $(tail -1 $O/bench_c4_$v.log | cut -c1-150)"
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
