# Round 5f: the candidate-overflow search (tools/cand_overflow_search.py) -> profiles/r05f_cand_overflow_search.txt.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python -u tools/cand_overflow_search.py > $O/ncand.txt 2>&1
cat $O/ncand.txt
