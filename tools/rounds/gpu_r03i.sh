# Round 3i: SIFT blur staging with batched loads + closed-form reflect, branch-free extrema test:
# SIFT parity tests, c1img line, c1img kernel trace.  -> gpurun_out/r03i/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests/test_sift_gpu.py tests/test_pipeline_gpu.py tests/test_dataset_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_sift.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -3 $O/pytest_sift.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
bash tools/prof_round.sh c1img > $O/prof_c1img.log 2>&1
echo done
