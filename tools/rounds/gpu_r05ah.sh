# Round 5ah: the prescreen with the problem's points staged in LDS (the point loop was global-load bound:
# cand kernel 0.12 -> 0.52 ms per C4 step in r05ag): GPU tests, then C4 / C3 against HEAD's library (no
# prescreen, variants/libmim_prev.so) and MIM_PRESCREEN=0, and c1img / dataset against HEAD, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prescreen or ransac or filtered or bound or configs or c3_full or pipeline or dataset or c4 or corpus or sift" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; k=r.get("kernel_ms_per_step_isolated") or r.get("kernel_ms_per_scene_isolated") or {}; print(d["value"], d["ms_per_step"], "exact", k.get("exact"), "cand", k.get("cand"), "single", d.get("single_scene_ms"))'; }
for i in 1 2; do
  for v in new prev off; do
    unset MIM_LIB MIM_PRESCREEN
    if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; fi
    if [ $v = off ]; then export MIM_PRESCREEN=0; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v: $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v: $(show $O/c3_${v}_$i.log)"
  done
done
unset MIM_PRESCREEN
for v in new prev; do
  unset MIM_LIB
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; fi
  timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_$v.log 2>&1; echo "c1img $v: $(show $O/c1img_$v.log)"
  timeout -k 10 300 python -u bench.py --config dataset --cpu-sample 0 --parity-sample 0 > $O/dataset_$v.log 2>&1; echo "dataset $v: $(show $O/dataset_$v.log)"
done
