# Round 6 ag: Barrett reduction of the attempt kernel with the full-rate v_mul_u32_u24 (was a mask and the
# quarter-rate v_mul_lo_u32): RANSAC and sampler GPU tests, C4 isolated sampler times against the
# previous commit's library -> profiles/r06ag_*
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ag
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_bounds_corpus_gpu.py tests/test_configs_gpu.py tests/test_small_sampler_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  MIM_LIB=$V/libmim_prev.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/prev_$i.log 2>&1
  echo "prev run $i: $(show $O/prev_$i.log)" | tee -a $O/summary.txt
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/new_$i.log 2>&1
  echo "new run $i: $(show $O/new_$i.log)" | tee -a $O/summary.txt
done
