# Widened bounds corpus (tests/test_bounds_corpus_gpu.py) at the default seeds, then at $1 seeds per family.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/corpus
timeout -k 10 600 python -u -m pytest tests/test_bounds_corpus_gpu.py -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/corpus/default.log 2>&1
rc=$?; echo "default rc=$rc"; grep -E "bounds corpus|passed|failed" gpurun_out/corpus/default.log | tail -4
[ $rc -eq 0 ] || exit $rc
MIM_CORPUS_SEEDS=${1:-200} timeout -k 10 900 python -u -m pytest tests/test_bounds_corpus_gpu.py -v -s --timeout 850 --timeout-method thread -p no:cacheprovider > gpurun_out/corpus/wide.log 2>&1
rc=$?; echo "wide rc=$rc"; grep -E "bounds corpus|passed|failed" gpurun_out/corpus/wide.log | tail -4
