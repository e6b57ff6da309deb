# Round 5am: the refine's LM loop takes the trial step's cost from the normal-equation pass at x - d
# (MIM_LM_MERGE, one pass over the inliers per iteration instead of two), and the refit's LtL sums read
# the inliers' L rows from LDS (MIM_LTL_STAGE).  Refine phase timing of
# c1img's slow problems (variants/libmim_rt.so, MIM_REFINE_TIMING), the pipeline / ransac GPU tests,
# then c1img with the merge on (lib) and off (variants/libmim_nomerge.so), two rounds, and C4 once each.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05am
mkdir -p $O
for v in rt0 rt; do
  MIM_LIB=variants/libmim_$v.so timeout -k 10 300 python -u bench.py --config c1img --steps 4 --warmup 1 --cpu-sample 0 --parity-sample 0 > $O/$v.log 2>&1 || true
  echo "$v: $(grep -c 'refine-timing' $O/$v.log || true) slow problems"
  grep "refine-timing" $O/$v.log | sort -t= -k6 -n -r | head -8 || true
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipeline or ransac or refine or dataset or c1img or configs" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; k=r.get("kernel_ms_per_step_isolated") or r.get("kernel_ms_per_scene_isolated") or {}; print(d["value"], d["ms_per_step"], "refine", k.get("refine"), "single", d.get("single_scene_ms"), "parity", (d.get("parity") or {}).get("mismatch"))'; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_on_$i.log 2>&1; echo "c1img merge on: $(show $O/c1img_on_$i.log)"
  MIM_LIB=variants/libmim_nomerge.so timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_off_$i.log 2>&1; echo "c1img merge off: $(show $O/c1img_off_$i.log)"
done
timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_on.log 2>&1; echo "c4 merge on: $(show $O/c4_on.log)"
MIM_LIB=variants/libmim_nomerge.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_off.log 2>&1; echo "c4 merge off: $(show $O/c4_off.log)"
