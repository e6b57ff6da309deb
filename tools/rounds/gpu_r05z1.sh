# Round 5 closing tree, part 1: the whole GPU suite and smoke, then three default bench runs each of C4
# (the driver's line), C3 and C5 -> profiles/r05_pytest_gpu.log, r05_smoke.log, r05_bench_<config>_<i>.log.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R05Z_OUT:-r05z}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"], "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)'; }
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/bench_c4_$i.log 2>&1; echo "c4 $(show $O/bench_c4_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --config c3 > $O/bench_c3_$i.log 2>&1; echo "c3 $(show $O/bench_c3_$i.log)"
  timeout -k 10 400 python -u bench.py --config c5 > $O/bench_c5_$i.log 2>&1; echo "c5 $(show $O/bench_c5_$i.log)"
done
