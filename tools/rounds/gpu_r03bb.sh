# Round 3bb: VALU issue rate per SIMD at 1-8 waves (tools/valu_rate_probe.hip), then SQ counters of the
# bound and distance kernels on one C3 step (two --pmc passes).  -> gpurun_out/r03bb/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bb
mkdir -p $O
timeout -k 10 120 ./tools/valu_rate_probe > $O/valu_rate.txt 2>&1
cat $O/valu_rate.txt
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex 'ransac_bound_mfma|knn2_i8' \
    -d $O/p$i -o run -- python3 bench.py --config c3 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $O/p$i.log 2>&1
done
python3 tools/pmc_summary.py $O > $O/summary.txt
grep -E "SQ_|GRBM|dispatch ms" $O/summary.txt | grep -E "bound|knn2_i8"
