# Round 3bf: closing checks and lines on the final tree: pytest -m gpu as the driver runs it, smoke, the
# bench lines (c4 default, c3, c5, c1img).  -> gpurun_out/r03bf/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bf
mkdir -p $O
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.log 2>&1
timeout -k 10 400 python -u bench.py --config c1img > $O/bench_c1img.log 2>&1
for f in c4 c3 c5 c1img; do tail -1 $O/bench_$f.log | cut -c1-220; done
