# Round 4p: (new) the check kernel gathering the sample points from LDS (the problem staged per block
# when n <= 2048) against the previous commit (prev), and the distance kernel's keyed early tiles
# (MIM_KNN_EARLY = 4 in prev, 6, 8, both built from the previous commit): pytest -m gpu, same-box
# alternating C4 lines, C3 lines, 8 problems of each against the oracle, kernel trace of the new tree.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
lib() { case $1 in new) unset MIM_LIB;; *) export MIM_LIB=$PWD/variants/libmim_$1.so;; esac; }
for rep in 1 2; do
  for v in new prev early6 early8; do
    lib $v
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 8 > $O/c4_${v}_$rep.log 2>&1
    echo "c4 $v $(tail -1 $O/c4_${v}_$rep.log | cut -c95-150)"
  done
done
for v in new prev early8; do
  lib $v
  timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 8 > $O/c3_$v.log 2>&1
  echo "c3 $v $(tail -1 $O/c3_$v.log | cut -c95-150)"
done
unset MIM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
