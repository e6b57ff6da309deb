# Round 4 closing tree (after the diamond bound), part 1: pytest -m gpu, smoke, and three runs each of
# the C4 (default) and C3 lines; the first C4 run with the default CPU sample (cpu_baseline).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c4_1.log 2>&1
for i in 2 3; do timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$i.log 2>&1; done
for i in 1 2 3; do timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3_$i.log 2>&1; done
for f in $O/bench_c4_*.log $O/bench_c3_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
