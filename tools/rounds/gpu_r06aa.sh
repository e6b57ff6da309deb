# Round 6 aa: deferred check attempts decided by their own kernel from per-round lists (VERDICT r05
# item 6): the RANSAC GPU tests and the corpus, then the C4 isolated sampler times against the previous
# commit's library (tools/build_prev.sh -> variants/libmim_prev.so) -> profiles/r06aa_*
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_bounds_corpus_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  MIM_LIB=$PWD/computervision_objectdetection_featurematching_amd/lib/variants/libmim_prev.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/prev_$i.log 2>&1
  echo "prev run $i: $(show $O/prev_$i.log)" | tee -a $O/summary.txt
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/new_$i.log 2>&1
  echo "new run $i: $(show $O/new_$i.log)" | tee -a $O/summary.txt
done
