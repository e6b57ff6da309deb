# The -m gpu suite, then the bounds corpus at $1 seeds per family (tests/test_bounds_corpus_gpu.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/corpus
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/corpus/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/corpus/suite.log
[ $rc -eq 0 ] || exit $rc
MIM_CORPUS_SEEDS=${1:-1000} timeout -k 10 1000 python -u -m pytest tests/test_bounds_corpus_gpu.py -v -s --timeout 950 --timeout-method thread -p no:cacheprovider > gpurun_out/corpus/big.log 2>&1
rc=$?; echo "big rc=$rc"; grep -E "bounds corpus|passed|failed" gpurun_out/corpus/big.log | tail -3
