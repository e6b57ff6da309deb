# Round 3v: DPP moves without a materialised old value (mov_dpp, bound_ctrl) in the group Jacobi /
# reductions vs update_dpp(0, ...) (variant dppold): RANSAC parity tests, isolated kernels (knn_ab:
# exact, refine), c1img line.  -> gpurun_out/r03v/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
set +e
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py tests/test_small_sampler_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MIM_LIB=$PWD/$V/libmim_dppold.so timeout -k 10 240 python -u tools/knn_ab.py --tag dppold --save > $O/ab.log 2> $O/ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag movdpp >> $O/ab.log 2>> $O/ab.err
MIM_LIB=$PWD/$V/libmim_dppold.so timeout -k 10 240 python -u tools/knn_ab.py --tag dppold2 >> $O/ab.log 2>> $O/ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag movdpp2 >> $O/ab.log 2>> $O/ab.err
python3 - <<'PY'
import json
for l in open("gpurun_out/r03v/ab.log"):
    d = json.loads(l); k = d["c3_kernels"]
    print(d["tag"], "exact", k["exact"], "refine", k["refine"], "chain", k["chain"], "step", d["c3_step_ms"], d["parity"][:40])
PY
