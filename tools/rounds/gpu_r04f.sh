# Round 4f: redraw lengths resolved in the attempt kernel, one thread per repeated-index position of
# the block from the LDS-staged draws (the irr kernel lists again, no stream reads): pytest -m gpu,
# C4 line, kernel trace, SQ counters of the sampler kernels; then the first-chunk A/B (4096 / 2048).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
K='ransac_attempt|ransac_check|ransac_irr|ransac_walk|ransac_count'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d $O/pmc$i -o run -- python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/pmc$i.log 2>&1
done
for fc in 2048; do
  MIM_FIRST_CHUNK=$fc MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c4 --steps 1 --warmup 0 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand_c4_fc$fc.log 2>&1
  MIM_FIRST_CHUNK=$fc timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_fc$fc.log 2>&1
  echo "fc=$fc $(tail -1 $O/bench_c4_fc$fc.log | cut -c1-160)"
done
MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c4 --steps 1 --warmup 0 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand_c4_fc4096.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_b.log 2>&1
echo "default again $(tail -1 $O/bench_c4_b.log | cut -c1-160)"
