# Round 5an: MIM_WINNER_H=1 (the settle pass also sends each chunk's first largest decided candidate
# through the exact pass, so its fp64 H reaches best_h and the refine skips its own runKernel): GPU
# parity tests with the knob on, then c1img (single scene) and C4 with it on and off, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05an
mkdir -p $O
MIM_WINNER_H=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prescreen or ransac or filtered or pipeline or dataset or c4 or c3_full or corpus or configs" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; k=r.get("kernel_ms_per_step_isolated") or r.get("kernel_ms_per_scene_isolated") or {}; print(d["value"], d["ms_per_step"], "exact", k.get("exact"), "refine", k.get("refine"), "single", d.get("single_scene_ms"), "parity", (d.get("parity") or {}).get("mismatch"))'; }
for i in 1 2; do
  for v in 1 0; do
    MIM_WINNER_H=$v timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_${v}_$i.log 2>&1; echo "c1img winner_h=$v: $(show $O/c1img_${v}_$i.log)"
  done
done
for v in 1 0; do
  MIM_WINNER_H=$v timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_$v.log 2>&1; echo "c4 winner_h=$v: $(show $O/c4_$v.log)"
done
