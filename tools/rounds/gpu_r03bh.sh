# Round 3bh: diagnose the x-half prefilter mismatch (tools/xpre_diff.py), candidate counts per chunk
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bh
mkdir -p $O
timeout -k 10 300 python -u tools/xpre_diff.py > $O/diff.log 2>&1
cat $O/diff.log | grep -v "^\[mim\]" | tail -20
