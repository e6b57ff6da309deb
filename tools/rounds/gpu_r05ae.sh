# Round 5ae: C4 candidate counts per chunk (MIM_DEBUG_NCAND) and the bound brackets against exact counts
# (MIM_CHECK_BOUNDS: width, tight fraction), one batch, for the exact pass's cost (r05ad).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ae
mkdir -p $O
MIM_DEBUG_NCAND=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand.log 2>&1 || true
grep "\[mim\] chunk" $O/ncand.log | sort | uniq -c | head -20
MIM_CHECK_BOUNDS=1 timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/bounds.log 2>&1 || true
grep "\[mim\] bound check" $O/bounds.log | head -8
