# Round GPU check: the -m gpu suite, then the default bench (C3) with its CPU baseline + parity.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.log 2>&1
echo "bench rc=$?"
tail -c 3000 gpurun_out/bench_c3.log
