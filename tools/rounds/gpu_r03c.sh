# Round 3c: the 32x32 distance kernel with the balanced schedule (default) + register-tile / stage /
# occupancy variants, parity tests, one PMC pair for the best candidate.  Output: gpurun_out/r03c/.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py tests/test_pipeline_gpu.py tests/test_ransac_gpu.py "tests/test_configs_gpu.py::test_c3_bounds_bracket_all_iterations" "tests/test_configs_gpu.py::test_batch_inlier_points_equals_per_problem_gather" "tests/test_configs_gpu.py::test_problem_detail_after_short_stream_reruns" "tests/test_configs_gpu.py::test_c5_dense_50k_sampled_rows" -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
for v in q4o2 q4o2s8 o2s8 q4o2w4 e2 q4nosel; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> $O/ab.log 2>> $O/ab.err
done
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for v in q4o2; do
  i=0
  for C in "$P1" "$P2"; do
    i=$((i+1))
    MIM_LIB=$PWD/$V/libmim_$v.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex knn2_i8 \
      -d $O/pmc_$v/p$i -o run -- python3 tools/knn_ab.py --tag $v --c3-only --steps 2 > $O/pmc_$v.p$i.log 2>&1
  done
  python3 tools/pmc_summary.py $O/pmc_$v > $O/pmc_$v.summary.txt
done
cat $O/ab.log
tail -2 $O/test.log
