# Round 4k: the distance kernel's dynamic schedule with each query-block sweep split into S train pieces
# (MIM_KNN_DYN_SPLIT, partial top-2 lists merged by the ratio kernel): shard-of-8 (32 problems per batch,
# 1.25 sweeps per resident block) and the full C4 batch at S = 1, 2, 4, alternating; 8 problems of each
# line checked against the oracle.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
for rep in 1 2; do
  for S in 1 2 4; do
    MIM_KNN_DYN_SPLIT=$S timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 8 --shard-of 8 > $O/s8_S${S}_$rep.log 2>&1
    echo "shard8 S=$S $(tail -1 $O/s8_S${S}_$rep.log | cut -c95-150)"
  done
done
for S in 1 2 4; do
  MIM_KNN_DYN_SPLIT=$S timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 8 > $O/c4_S${S}.log 2>&1
  echo "c4 S=$S $(tail -1 $O/c4_S${S}.log | cut -c95-150)"
done
for S in 1 2 4; do
  MIM_KNN_DYN_SPLIT=$S timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 8 --shard-of 4 > $O/s4_S${S}.log 2>&1
  echo "shard4 S=$S $(tail -1 $O/s4_S${S}.log | cut -c95-150)"
done
