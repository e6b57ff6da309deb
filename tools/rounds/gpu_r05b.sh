# Round 5b: MFMA forms beside VALU and role-split waves (tools/issue_probe.hip sections C, D).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 180 ./tools/issue_probe > $O/issue_probe.txt 2>&1
cat $O/issue_probe.txt
