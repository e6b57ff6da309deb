# Round 3bm: the N-rank bench path on the final tree, rehearsed on one GPU: 2 ranks over gloo (records
# gathered through host memory; the 8-GPU RCCL run is the driver's), and rank 0's shard of an 8-rank C4
# run (--shard-of 8).  -> gpurun_out/r03bm/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bm
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --cpu-sample 0 > $O/bench_c4_gloo2.log 2>&1
tail -1 $O/bench_c4_gloo2.log | cut -c1-300
timeout -k 10 300 python -u bench.py --shard-of 8 --steps 60 --cpu-sample 0 --iso-steps 2 > $O/bench_c4_shard_of_8.log 2>&1
tail -1 $O/bench_c4_shard_of_8.log | cut -c1-300
