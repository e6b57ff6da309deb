# Round 5ag: the candidate prescreen (cand kernel: closed-form disc test in fp64; MIM_PRESCREEN=1 default):
# its GPU test and the RANSAC / bound / config / pipeline / dataset tests, C4's decided fraction
# (MIM_DEBUG_NCAND), then C4 and C3 lines with the prescreen on and off, two interleaved rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prescreen or ransac or filtered or bound or configs or c3_full or pipeline or dataset or c4 or corpus" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MIM_DEBUG_NCAND=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --inflight 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 > $O/ncand.log 2>&1 || true
grep "\[mim\] chunk" $O/ncand.log | sort | uniq -c | head -6
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "exact", r["exact"], "cand", r["cand"], "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  for ps in 1 0; do
    MIM_PRESCREEN=$ps timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c4_ps${ps}_$i.log 2>&1; echo "c4 prescreen $ps: $(show $O/c4_ps${ps}_$i.log)"
    MIM_PRESCREEN=$ps timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 4 --iso-steps 2 > $O/c3_ps${ps}_$i.log 2>&1; echo "c3 prescreen $ps: $(show $O/c3_ps${ps}_$i.log)"
  done
done
