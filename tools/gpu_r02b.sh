# Round-2 GPU check after the distance-kernel rework: the -m gpu suite, bench lines C3 (default),
# C1-surrogate and C5, the rocprofv3 kernel-trace + stats of the default bench and the HBM PMC passes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02b/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r02b/pytest.log
[ $rc -eq 0 ] || exit $rc
for C in c3 c1 c5; do
  timeout -k 10 300 python -u bench.py --config $C > gpurun_out/r02b/bench_$C.log 2>&1 || { echo "bench $C rc=$?"; exit 1; }
  echo "bench $C ok"; tail -n 1 gpurun_out/r02b/bench_$C.log | cut -c 1-400
done
bash tools/prof_bench.sh || { echo "prof_bench failed"; exit 1; }
bash tools/prof_round.sh || { echo "prof_round failed"; exit 1; }
echo profiles done
