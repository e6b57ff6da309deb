# Round 5l: the latency kernels' footprint beside the batches in flight: refine with one problem per block
# (MIM_REFINE_RW=1: 12.6 KB LDS per block instead of 50 KB) and the chain walk on 512 threads with a
# 4,096-entry LDS piece (MIM_WALK_THREADS / _ENTRIES: 23 KB instead of 43 KB, 8 waves instead of 16):
# RANSAC tests per variant, then C4 and the 32-problem shard A/B, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
for v in both; do
  MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_configs_gpu.py tests/test_small_sampler_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -5 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "refine", r.get("refine"), "chain", r.get("chain"))'; }
for i in 1 2; do
  for v in base rw1 walk512 both; do
    if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/$V/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
  done
done
for v in base both; do
  if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/$V/libmim_$v.so; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 > $O/s8_$v.log 2>&1; echo "s8 $v $(show $O/s8_$v.log)"
done
