# Round 4 closing tree (after the diamond bound), part 3: rocprofv3 kernel traces (and HBM counter passes) of C5 and c1img
# (tools/prof_round.sh), and the distance and bound kernels' SQ counters on C4 (two passes).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z4
mkdir -p $O
for c in c5 c1img; do timeout -k 10 900 bash tools/prof_round.sh $c; done
K='knn2_i8|ransac_bound_mfma'
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d $O/pmc_sq$i -o run -- python3 bench.py --inflight 1 --steps 2 --warmup 1 --iso-steps 1 --cpu-sample 0 > $O/pmc_sq$i.log 2>&1
done
