# Round 5d: packed-f32 issue costs (tools/issue_probe.hip, section A) and point sets that overflow the
# RANSAC candidate list without MIM_CAND_CAP ((an earlier version of tools/cand_overflow_search.py)).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 180 ./tools/issue_probe > $O/issue_probe.txt 2>&1
head -30 $O/issue_probe.txt
timeout -k 10 300 python -u (an earlier version of tools/cand_overflow_search.py) > $O/ncand.txt 2>&1
cat $O/ncand.txt
