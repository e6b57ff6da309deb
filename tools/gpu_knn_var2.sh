# Distance-kernel iteration: the -m gpu suite on the default build, then for every variant in
# lib/variants: kNN parity tests + the C3 and C5 bench lines (no CPU sample).  Logs: gpurun_out/var/.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/var/suite_default.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/var/suite_default.log
[ $rc -eq 0 ] || exit $rc
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  MIM_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/var/$n.test 2>&1
  rc=$?; echo "$n test rc=$rc"; tail -1 gpurun_out/var/$n.test
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  for c in c3 c5; do
    MIM_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 1 --cpu-sample 0 > gpurun_out/var/$n.$c.bench 2>&1 || { echo "$n bench $c failed"; exit 1; }
    python3 - gpurun_out/var/$n.$c.bench <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "knn ms", r.get("kernel_ms_per_step", {}).get("knn"),
      "iso", r.get("isolated_kernel_ms_per_step", {}).get("knn"), "frac", r["frac"], "iso_frac", r.get("isolated_frac"))
PY
  done
done
