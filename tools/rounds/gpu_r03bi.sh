# Round 3bi: the scenes-in-flight pipeline test, 3x with the x-half prefilter and 3x without
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bi
mkdir -p $O
for rep in 1 2 3; do
  for X in 1 0; do
    MIM_BOUND_XPRE=$X timeout -k 10 200 python -u -m pytest tests/test_pipeline_gpu.py -q -k in_flight --timeout 150 --timeout-method thread > $O/t_${X}_$rep.log 2>&1
    echo "xpre=$X rep $rep rc $?: $(tail -1 $O/t_${X}_$rep.log)"
    grep -E "^E\s+4_|Mismatched" $O/t_${X}_$rep.log | head -2
  done
done
