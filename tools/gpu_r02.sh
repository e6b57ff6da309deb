# Round-2 GPU check: the -m gpu suite, then the bench lines of C3 (default), C1-surrogate and C5.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for C in c3 c1 c5; do
  timeout -k 10 240 python -u bench.py --config $C > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C rc=$?"; exit 1; }
  echo "bench $C ok"
  tail -n 1 gpurun_out/bench_$C.log | cut -c 1-600
done
