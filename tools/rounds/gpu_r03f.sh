# Round 3f: XCD-aware distance-kernel chunk placement (parity tests, C3/C5 timing, C3 HBM counters),
# SIFT scales back on one stream (c1img line; per-scale streams as the A/B).  -> gpurun_out/r03f/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py tests/test_sift_gpu.py tests/test_pipeline_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/knn_ab.py --tag xcd > $O/ab.log 2> $O/ab.err
cut -c1-300 $O/ab.log
timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
MIM_SIFT_SCALE_STREAMS=1 timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_c1img_streams.log 2>&1
tail -1 $O/bench_c1img_streams.log | cut -c1-300
bash tools/prof_round.sh c3 > $O/prof_c3.log 2>&1
cat gpurun_out/prof_c3/pmc_traffic.json | head -12
