# Round 5a: instruction issue costs (tools/issue_probe.hip: single VALU ops at 8 waves per SIMD, MFMA
# beside VALU at 1/2/4 waves per SIMD) and the round-start C4 line on this box.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 120 ./tools/issue_probe > $O/issue_probe.txt 2>&1
cat $O/issue_probe.txt
timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-400
