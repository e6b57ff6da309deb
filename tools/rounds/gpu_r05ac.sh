# Round 5ac: one library call for a step's scene sets (mim_sets_create / Matcher.add_sets): its GPU test
# and the sets tests, then host enqueue per step and the C4 line at the default and the 20-step window,
# and the 32-problem shard.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sets_truncate_gpu.py tests/test_c4_rccl_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "host", d["host_enqueue_ms_per_step"])'; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 1 > $O/c4_$i.log 2>&1; echo "c4 k60: $(show $O/c4_$i.log)"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --parity-sample 0 --iso-steps 1 > $O/c4_k20_$i.log 2>&1; echo "c4 k20: $(show $O/c4_k20_$i.log)"
  timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 --parity-sample 0 --iso-steps 1 > $O/s8_$i.log 2>&1; echo "s8: $(show $O/s8_$i.log)"
done
