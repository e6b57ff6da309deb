# Round 5m: the bound kernel's prologue with 6 fp64 divisions instead of 13 (sa, sb are powers of two;
# square_to_quad's two quotients by one reciprocal): bound bracket / filtered == exact / corpus tests, then a
# C4 A/B against HEAD's ransac.hip (bound kernel time per step), two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "bound or filtered or corpus or c3_full or candidate" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "score", r["kernel_ms_per_step_isolated"]["score"], "exact", r["kernel_ms_per_step_isolated"]["exact"], r["others"]["bound"]["issue_model"])'; }
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
  done
done
