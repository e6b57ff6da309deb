# Round 5ao: MIM_WINNER_H on by default for problems of fewer than 256 good matches (real SIFT views):
# the GPU suite, then three c1img and dataset lines (closing numbers for the scene configs) and one C4
# line (its problems are above the limit: unchanged path).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; k=r.get("kernel_ms_per_step_isolated") or r.get("kernel_ms_per_scene_isolated") or {}; print(d["value"], d["ms_per_step"], "refine", k.get("refine"), "single", d.get("single_scene_ms"), "scenes/s", d.get("scenes_per_s"), "parity", (d.get("parity") or {}).get("mismatch"))'; }
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --config c1img > $O/bench_c1img_$i.log 2>&1; echo "c1img $(show $O/bench_c1img_$i.log)"
  timeout -k 10 400 python -u bench.py --config dataset > $O/bench_dataset_$i.log 2>&1; echo "dataset $(show $O/bench_dataset_$i.log)"
done
timeout -k 10 400 python -u bench.py > $O/bench_c4_1.log 2>&1; echo "c4 $(show $O/bench_c4_1.log)"
