# Round 5w: the distance kernel with a 3-deep LDS ring and per-buffer LDS counters instead of a block
# barrier per stage (MIM_KNN_RING=1, 3-tile stages: variants/libmim_ring.so), VERDICT r04 item 2's first
# candidate.  kNN GPU tests on the variant first (bit-identical rows), then isolated launch and pipelined
# lines against the default (4-tile stages, barrier) and 3-tile stages with the barrier (libmim_st3.so).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
export MIM_LIB=$PWD/variants/libmim_ring.so
timeout -k 10 120 python -u -m pytest tests/test_knn_gpu.py -x -q --timeout 100 --timeout-method thread -k "sift_exact" > $O/pytest_ring_first.log 2>&1 || { tail -30 $O/pytest_ring_first.log; exit 1; }
tail -1 $O/pytest_ring_first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or configs or c3_full or dataset or c5" > $O/pytest_ring.log 2>&1 || { tail -30 $O/pytest_ring.log; exit 1; }
tail -1 $O/pytest_ring.log
unset MIM_LIB
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"])'; }
for i in 1 2; do
  for v in base ring st3; do
    if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c5 --cpu-sample 0 --parity-sample 0 > $O/c5_${v}_$i.log 2>&1; echo "c5 $v $(show $O/c5_${v}_$i.log)"
  done
done
