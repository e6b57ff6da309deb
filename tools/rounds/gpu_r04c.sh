# Round 4c: why the sampler kernels (attempt, irr, walk, check, count) take ~1.8 ms per C4 step when
# their VALU and byte counts say ~0.2: kernel trace of one isolated C4 batch + SQ counters per kernel.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
K='ransac_attempt|ransac_check|ransac_irr|ransac_walk|ransac_count'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d $O/pmc$i -o run -- python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/pmc$i.log 2>&1
done
