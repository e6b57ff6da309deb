# Round 3bs: Jacobi pivot as three 32-bit DPP passes (|p| high/low words, then the smallest packed key),
# on top of r03br: pytest -m gpu (H bits vs the oracle), smoke, then c1img / C3 / C4 lines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bs
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --config c1img > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.log 2>&1
tail -1 $O/bench_c3.log | cut -c1-300
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-300
