# RANSAC-kernel iteration: for every variant in lib/variants: the RANSAC + bounds-corpus GPU tests and
# the C3 bench line (no CPU sample), isolated per-kernel times printed.  Logs: gpurun_out/vr/.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/vr
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  MIM_LIB=$PWD/$so timeout -k 10 400 python -u -m pytest tests/test_ransac_gpu.py tests/test_bounds_corpus_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/vr/$n.test 2>&1
  rc=$?; echo "$n test rc=$rc"; tail -1 gpurun_out/vr/$n.test
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  MIM_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 1 --cpu-sample 0 > gpurun_out/vr/$n.bench 2>&1 || { echo "$n bench failed"; exit 1; }
  python3 - gpurun_out/vr/$n.bench <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "iso", {k: v for k, v in r.get("isolated_kernel_ms_per_step", {}).items() if v})
PY
done
