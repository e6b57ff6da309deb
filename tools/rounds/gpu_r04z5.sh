# Round 4 closing tree (after the diamond bound), part 2: three runs each of C5, c1img and the reference's whole dataset run, then
# the rocprofv3 kernel traces and HBM counter passes of C4 and C3 (tools/prof_round.sh).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z4
mkdir -p $O
for c in c5 c1img dataset; do
  for i in 1 2 3; do timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 > $O/bench_${c}_$i.log 2>&1; done
done
for f in $O/bench_c5_*.log $O/bench_c1img_*.log $O/bench_dataset_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
for c in c4 c3; do timeout -k 10 900 bash tools/prof_round.sh $c; done
