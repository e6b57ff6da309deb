# Round 6 v: the adversarial corpus with four new families (pythag, scales, two_models, dups): every
# bracket against the exact count, filtered == all-exact, prescreen decisions recounted
# -> profiles/r06v_pytest_corpus.log
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bounds_corpus_gpu.py tests/test_ransac_gpu.py -m gpu -x -v -s --timeout 500 --timeout-method thread > $O/pytest_corpus.log 2>&1 || { tail -60 $O/pytest_corpus.log; exit 1; }
grep -E "corpus|passed|failed" $O/pytest_corpus.log | tail -8
