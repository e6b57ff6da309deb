# Round 6 ae: the check kernel's deferred attempts through ransac_check_defer_kernel (final form): the
# RANSAC, corpus, config and pipeline GPU tests -> profiles/r06ae_pytest.log
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
