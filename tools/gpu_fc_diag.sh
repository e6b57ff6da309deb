# diagnose the first-chunk-512 mismatch: the c1 surrogate test under sampler / selection modes
cd $GRAFT_REPO_ROOT
for mode in "MIM_SAMPLER_STREAM=0" "MIM_SAMPLER_WALK=1" "MIM_RANSAC_EXACT=1" "MIM_FIRST_CHUNK=2000"; do
  env MIM_FIRST_CHUNK=512 $mode timeout -k 10 200 python -u -m pytest tests/test_configs_gpu.py -x -q -k c1_surrogate --timeout 180 --timeout-method thread > "gpurun_out/fc_$mode.log" 2>&1
  rc=$?; echo "$mode rc=$rc $(tail -1 "gpurun_out/fc_$mode.log")"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
