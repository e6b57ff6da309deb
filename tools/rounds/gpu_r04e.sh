# Round 4e: first-chunk size A/B on C4 (MIM_FIRST_CHUNK 4096 default vs 2048 / 1024): chunk 1 runs the
# bound kernel with the lower bound (10 VALU per pair), chunk 2 without (4); a shorter chunk 1 leaves a
# lower maxGoodCount, so more chunk-2 candidates for the exact kernel.  Candidates per chunk logged.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
for fc in 4096 2048 1024; do
  MIM_FIRST_CHUNK=$fc MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c4 --steps 1 --warmup 0 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand_c4_fc$fc.log 2>&1
  MIM_FIRST_CHUNK=$fc timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_fc$fc.log 2>&1
  echo "fc=$fc $(tail -1 $O/bench_c4_fc$fc.log | cut -c1-160)"
done
