# Round 5q: the distance kernel's late tiles software-pipelined over half tiles (next half tile's A
# fragments and parity word read from LDS right after this one's MFMAs; MIM_KNN_PREFETCH=1): kNN GPU tests,
# then C4 / C3 / C5 and the 32-problem shard A/B against HEAD's knn.hip (variants/libmim_prev.so), two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or configs or c3_full or dataset" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"])'; }
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c5 --cpu-sample 0 --parity-sample 0 > $O/c5_${v}_$i.log 2>&1; echo "c5 $v $(show $O/c5_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 --parity-sample 0 > $O/s8_${v}_$i.log 2>&1; echo "s8 $v $(show $O/s8_${v}_$i.log)"
  done
done
