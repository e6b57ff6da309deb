# r06a: distance-kernel breakdown.  (1) the gfx950 counter list; (2) C3-shape isolated launch of the
# probe builds (no events / no filter / no seeds) and the candidate fixes, two interleaved rounds;
# parity of the candidate fixes against the base build; (3) wait/issue counters of knn2_i8 on C4.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
MIM_LIB=$PWD/$V/libmim_base.so timeout -k 10 300 python3 -u tools/knn_ab.py --tag base --save --steps 10 > $O/ab_base_full.json 2> $O/ab_base_full.err
for v in pw prio pwprio; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 300 python3 -u tools/knn_ab.py --tag $v --steps 10 > $O/ab_${v}_full.json 2> $O/ab_${v}_full.err
done
for i in 1 2; do
  for v in base p1 p2 p3 pw prio pwprio; do
    MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python3 -u tools/knn_ab.py --tag $v --c3-only --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err
  done
done
# counters of the base build on C4 (isolated batches), one pass per line (<= 8 SQ counters each)
i=0
while read -r P; do
  i=$((i+1))
  MIM_LIB=$PWD/$V/libmim_base.so timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv --kernel-include-regex knn2_i8 \
    -d $O/pmc/p$i -o run -- python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/pmc_p$i.log 2>&1 < /dev/null
done <<'PASSES'
GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES
GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_IFETCH
GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL
GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_FLAT SQ_IFETCH_LEVEL SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_WAVES
PASSES
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
timeout -k 10 300 python3 -u -m pytest tests/test_group.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_group.log 2>&1 || echo "group test failed"
timeout -k 10 600 python3 -u -m pytest tests/test_ransac_gpu.py tests/test_small_sampler_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_ransac.log 2>&1 || echo "ransac tests failed"
echo done
