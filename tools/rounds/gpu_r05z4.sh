# Round 5 closing tree, part 4 (final tree after the bench's traffic / queue-default changes): the whole
# GPU suite and smoke once more, and the 2-rank launcher with both ranks on the one GPU (gloo record
# gather) -> profiles/r05_pytest_gpu_final.log, r05_bench_c4_gloo2.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R05Z4_OUT:-r05z4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_final.log 2>&1 || { tail -40 $O/pytest_gpu_final.log; exit 1; }
tail -1 $O/pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_final.log 2>&1
tail -1 $O/smoke_final.log
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 8 --cpu-sample 0 > $O/bench_c4_gloo2.log 2>&1
tail -1 $O/bench_c4_gloo2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["n_gpus"], d.get("ranks_seen"), d["gather"]["records"], d["gather"]["status_counts"], d["parity"])'
