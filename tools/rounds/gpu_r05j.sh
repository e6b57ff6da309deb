# Round 5j: distance kernel with one 16-wave block per CU (1,024 queries per staged tile: half the LDS-DMA
# bytes and barriers per MFMA), stages of 4 or 8 tiles (MIM_KNN_WAVES=16, MIM_KNN_STAGE=8 variants,
# tools/build_variants.sh): kNN tests per variant, then C4 / C3 / C5 A/B on one box.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
for v in w16 w16s8; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_golden_gpu.py -m gpu -x -q -k "not split_tail" --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -5 $O/pytest_$v.log; }
  tail -1 $O/pytest_$v.log
done
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r.get("launch_ms"), r.get("frac"))'; }
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -m gpu -x -q -k split_tail --timeout 250 --timeout-method thread > $O/pytest_tail.log 2>&1 || { tail -20 $O/pytest_tail.log; exit 1; }
tail -1 $O/pytest_tail.log
for i in 1 2; do
  for v in base w16 w16s8; do
    if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/$V/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
  done
done
for v in base w16 w16s8; do
  if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/$V/libmim_$v.so; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c3 > $O/c3_$v.log 2>&1; echo "c3 $v $(show $O/c3_$v.log)"
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c5 > $O/c5_$v.log 2>&1; echo "c5 $v $(show $O/c5_$v.log)"
done
