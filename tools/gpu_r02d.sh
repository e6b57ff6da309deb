# Round-2 closing GPU check after the small-problem sampler, fused blur and set truncation: the -m gpu suite, bench lines
# C3 (default), C1 surrogate, C1 on the reference's images, C5, the rocprofv3 kernel trace + stats of
# the default bench (prof_bench.sh) and of the SIFT timing script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02d/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r02d/pytest.log
[ $rc -eq 0 ] || exit $rc
for C in c3 c1 c1img c5; do
  timeout -k 10 300 python -u bench.py --config $C > gpurun_out/r02d/bench_$C.log 2>&1 || { echo "bench $C rc=$?"; exit 1; }
  echo "bench $C ok"; tail -n 1 gpurun_out/r02d/bench_$C.log | cut -c 1-300
done
timeout -k 10 120 python tools/time_sift.py --oracle > gpurun_out/r02d/time_sift.json 2>/dev/null || exit 1
bash tools/prof_bench.sh || { echo "prof_bench failed"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/prof_sift -o run --output-format csv -- python3 tools/time_sift.py --reps 3 > gpurun_out/r02d/prof_sift.log 2>&1 || { echo "prof_sift failed"; exit 1; }
echo prof-done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/run_dataset.py > gpurun_out/r02d/dataset_run.json 2>gpurun_out/r02d/dataset_run.err || { echo "dataset failed"; exit 1; }
timeout -k 10 120 python -u tools/walk_probe.py > gpurun_out/r02d/walk_probe.log 2>&1 || exit 1
echo all-done
