# Round 5h: the distance kernel's split tail (api.cpp, MIM_KNN_TAIL) and the sampler kernels' XCD placement
# and grid floor (ransac.hip): whole GPU suite + smoke on the new tree, then same-box A/B at the 8-GPU
# shard (--shard-of 8), the full C4 batch and C3: new = both, tail = the split tail alone, prev = HEAD.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; k=r["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "knn", k["knn"], "score", k["score"], "attempt", k["attempt"], "check", k["check"])'; }
for i in 1 2; do
  for v in new tail prev; do
    if [ $v != new ]; then export MIM_LIB=$PWD/variants/libmim_$v.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 > $O/bench_c4s8_${v}_$i.log 2>&1
    echo "c4 shard-of-8 $v $(show $O/bench_c4s8_${v}_$i.log)"
  done
done
for v in new prev; do
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "c4 $v $(show $O/bench_c4_$v.log)"
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c3 > $O/bench_c3_$v.log 2>&1
  echo "c3 $v $(show $O/bench_c3_$v.log)"
done
