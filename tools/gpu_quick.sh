# Quick GPU check: selected tests ($1, pytest -k expression), then the default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$1" > gpurun_out/pytest_quick.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
shift
for cfg in "$@"; do
  timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || exit $?
  echo "bench $cfg ok"; tail -c 2500 gpurun_out/bench_$cfg.log; echo
done
