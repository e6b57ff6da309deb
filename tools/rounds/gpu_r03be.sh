# Round 3be: profiles of the closing distance kernel (keyed early tiles, scalar candidate masks):
# tools/prof_round.sh per config (isolated kernel trace + stats, FETCH/WRITE passes).  -> gpurun_out/prof_*
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in c4 c3 c5 c1img; do
  bash tools/prof_round.sh $C > gpurun_out/prof_$C.log 2>&1 || { echo "prof $C failed"; tail -5 gpurun_out/prof_$C.log; exit 1; }
  echo "prof $C done"; tail -1 gpurun_out/prof_$C/bench_trace.log | cut -c1-200
done
