# Round 3bg: chunk-2 bounds by the x-half prefilter + the box test of the listed iterations (default)
# vs the box test of every iteration (MIM_BOUND_XPRE=0): pytest -m gpu, per-kernel times (knn_ab C3),
# candidate counts, pipelined C4 / C3 alternating.  -> gpurun_out/r03bg/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03bg
mkdir -p $O
set +e
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit 1; fi
MIM_BOUND_XPRE=0 timeout -k 10 240 python -u tools/knn_ab.py --tag full --save --c3-only > $O/ab.log 2> $O/ab.err || true
for rep in 1 2; do
  timeout -k 10 200 python -u tools/knn_ab.py --tag xpre --c3-only >> $O/ab.log 2>> $O/ab.err || true
  MIM_BOUND_XPRE=0 timeout -k 10 200 python -u tools/knn_ab.py --tag full --c3-only >> $O/ab.log 2>> $O/ab.err || true
done
cat $O/ab.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d['c3_kernels']; print(d['tag'], 'score', k.get('score'), 'cand', k.get('cand'), 'exact', k.get('exact'), 'step', d.get('c3_step_ms'), d.get('parity','')[:20])"
MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c3 --steps 1 --warmup 0 --inflight 1 --cpu-sample 0 --iso-steps 0 > $O/ncand_xpre.log 2>&1 || true
MIM_BOUND_XPRE=0 MIM_DEBUG_NCAND=1 timeout -k 10 200 python -u bench.py --config c3 --steps 1 --warmup 0 --inflight 1 --cpu-sample 0 --iso-steps 0 > $O/ncand_full.log 2>&1 || true
grep -c "candidates mean" $O/ncand_xpre.log $O/ncand_full.log || true
diff <(grep "candidates mean" $O/ncand_xpre.log) <(grep "candidates mean" $O/ncand_full.log) > /dev/null && echo "candidate counts identical" || echo "candidate counts DIFFER"
for rep in 1 2; do
  for X in 1 0; do
    MIM_BOUND_XPRE=$X timeout -k 10 300 python -u bench.py --cpu-sample 0 --iso-steps 2 > $O/b.log 2>&1
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 xpre=$X', d['value'], d['ms_per_step'], d['roofline'].get('others',{}).get('bound',{}).get('launch_ms'))"
  done
done
