# Round 3br: Jacobi rotation with hypot(p, t) and p / t from one quotient (one fp64 division less per rotation),
# and the pivot candidates read branch-free, on top of r03bq: pytest -m gpu (H bits vs the oracle), then c1img / C3 / C4 lines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03br
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --config c1img > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.log 2>&1
tail -1 $O/bench_c3.log | cut -c1-300
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-300
