# Round 6 closing tree, part 1: the whole GPU suite and smoke, then three default bench runs of C4 (the
# driver's line) -> profiles/r06_pytest_gpu.log, r06_smoke.log, r06_bench_c4_<i>.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"], "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)'; }
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/bench_c4_$i.log 2>&1; echo "c4 $(show $O/bench_c4_$i.log)"
done
