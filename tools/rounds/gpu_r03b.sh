# Round 3b: distance-kernel variants (LDS prefetch, column-tile counts, occupancy, selection-free
# probes) + PMC passes, then the reworked bench (C4 default) end to end.  Output: gpurun_out/r03b_*.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
O=gpurun_out/r03b
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 500 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py tests/test_pipeline_gpu.py "tests/test_configs_gpu.py::test_batch_inlier_points_equals_per_problem_gather" "tests/test_configs_gpu.py::test_problem_detail_after_short_stream_reruns" tests/test_cpp_host.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
MIM_LIB=$PWD/$V/libmim_legacy.so timeout -k 10 240 python -u tools/knn_ab.py --tag legacy --save > $O/ab.log 2> $O/ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag pf4 >> $O/ab.log 2>> $O/ab.err
for v in pf0 ct3 ct2 ct4o2 nosel4 nosel2 legnosel; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 200 python -u tools/knn_ab.py --tag $v >> $O/ab.log 2>> $O/ab.err
done
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for v in default legacy nosel4; do
  lib=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
  [ $v != default ] && lib=$PWD/$V/libmim_$v.so
  i=0
  for C in "$P1" "$P2"; do
    i=$((i+1))
    MIM_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex knn2_i8 \
      -d $O/pmc_$v/p$i -o run -- python3 tools/knn_ab.py --tag $v --c3-only --steps 2 > $O/pmc_$v.p$i.log 2>&1
  done
  python3 tools/pmc_summary.py $O/pmc_$v > $O/pmc_$v.summary.txt
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 1 --cpu-sample 2 --cpu-rounds 1 > $O/bench_c4.log 2>&1
cat $O/ab.log
tail -1 $O/bench_c4.log | cut -c1-600
