# Round 6 closing tree, part 4: the round's kernel traces and HBM counters of C4, C3, C5 and c1img
# (tools/prof_round.sh) -> profiles/r06_kernel_stats_<config>.csv, r06_pmc_traffic_<config>.json.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in c4 c3 c5 c1img; do
  timeout -k 10 900 bash tools/prof_round.sh $C
  echo "prof $C done"
done
