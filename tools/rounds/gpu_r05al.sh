# Round 5al: the settle pass after the prescreen (undecided candidates whose upper bound cannot beat the
# decided counts listed before them are dropped; MIM_SETTLE=0: off): corpus diagnostic, GPU tests, then
# C4 / C3 with the settle pass on and off, and c1img / dataset, two rounds, plus C4's counts.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05al
mkdir -p $O
timeout -k 10 300 python -u tools/diag_prescreen.py > $O/corpus.log 2>&1 || true
echo "corpus recount mismatches: $(grep -c 'prescreen mismatch' $O/corpus.log || true)"; grep "differ:" $O/corpus.log || tail -5 $O/corpus.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prescreen or ransac or filtered or bound or configs or c3_full or pipeline or dataset or c4 or corpus or sift" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MIM_DEBUG_NCAND=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand.log 2>&1 || true
grep "\[mim\] chunk" $O/ncand.log | sort | uniq -c | head -4
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; k=r.get("kernel_ms_per_step_isolated") or r.get("kernel_ms_per_scene_isolated") or {}; print(d["value"], d["ms_per_step"], "exact", k.get("exact"), "cand", k.get("cand"), "single", d.get("single_scene_ms"), "parity", (d.get("parity") or {}).get("mismatch"))'; }
for i in 1 2; do
  for v in on off; do
    unset MIM_SETTLE
    if [ $v = off ]; then export MIM_SETTLE=0; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_${v}_$i.log 2>&1; echo "c4 settle $v: $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c3_${v}_$i.log 2>&1; echo "c3 settle $v: $(show $O/c3_${v}_$i.log)"
  done
done
unset MIM_SETTLE
timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_on.log 2>&1; echo "c1img settle on: $(show $O/c1img_on.log)"
timeout -k 10 300 python -u bench.py --config dataset --cpu-sample 0 --parity-sample 0 > $O/dataset_on.log 2>&1; echo "dataset settle on: $(show $O/dataset_on.log)"
