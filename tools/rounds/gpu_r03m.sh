# Round 3m: the round's profiles on the closing kernels: isolated kernel traces + HBM counters of
# C3 / C4 / C5 and the c1img trace (tools/prof_round.sh).  -> gpurun_out/prof_*/, gpurun_out/r03m/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
for C in c3 c4 c5 c1img; do
  bash tools/prof_round.sh $C > $O/prof_$C.log 2>&1
  echo "prof $C done"
done
