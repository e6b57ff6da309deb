# Round 3s: largest octave fused into the one-block small-octave kernel (MIM_SMALL_PLANE: 8192 default,
# 2048, 512): SIFT tests on the default, c1img line of each (sift_640x480_ms = one image's
# SIFT latency).  -> gpurun_out/r03s/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
for v in sp2048 sp512; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 600 python -u -m pytest tests/test_sift_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  tail -1 $O/pytest_$v.log || true
done
for v in default sp2048 sp512 default sp2048 sp512; do
  if [ $v = default ]; then L=""; else L=$PWD/$V/libmim_$v.so; fi
  MIM_LIB=$L timeout -k 10 400 python -u bench.py --config c1img --cpu-sample 0 > $O/bench_$v.log 2>&1
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['sift_640x480_ms'], d['single_scene_ms'])"
done
