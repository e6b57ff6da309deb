# Round 4b: chunk-2 bound A/B, box (default) vs disc (MIM_BOUND_DISC=1): candidate counts per chunk
# (MIM_DEBUG_NCAND) and the C3 / C4 lines; the sampler grids sized by the estimated window.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
for mode in 0 1; do
  MIM_BOUND_DISC=$mode MIM_DEBUG_NCAND=1 timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --inflight 1 --iso-steps 1 --cpu-sample 0 > $O/ncand_c3_disc$mode.log 2>&1
  grep -c "candidates" $O/ncand_c3_disc$mode.log
  MIM_BOUND_DISC=$mode timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4_disc$mode.log 2>&1
  tail -1 $O/bench_c4_disc$mode.log | cut -c1-200
done
