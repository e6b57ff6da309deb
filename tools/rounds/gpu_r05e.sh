# Round 5e: point sets that overflow the RANSAC candidate list without MIM_CAND_CAP (second search).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u (an earlier version of tools/cand_overflow_search.py) > $O/ncand.txt 2>&1
cat $O/ncand.txt
