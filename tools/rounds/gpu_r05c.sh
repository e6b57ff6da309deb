# Round 5c: the bound kernel's clamped float counts (fast-rate VALU instead of v_alignbit + v_bcnt):
# bound bracket / filtered == exact / corpus tests, the ADVICE fixes' tests (C++ Detector cache,
# device-set rows, find_homography message), then same-box A/B against the round-4 ransac.hip.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "bound or filtered or corpus or cpp_host or scales_sets_rows or find_homography_names or detect_objects_matches" \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in new prev new prev; do
  if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench_c4_$v.log 2>&1
  echo "c4 $v $(tail -1 $O/bench_c4_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("others",{}))' 2>&1 | cut -c1-400)"
done
unset MIM_LIB
