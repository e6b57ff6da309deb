# Round 5x: what the bound kernel spends outside its tile arithmetic: timing probes with the tile math
# compiled out (MIM_PROBE_BOUND=1: prologue + LDS staging + epilogue) and the whole tile loop compiled out
# (=2: prologue + epilogue), isolated per-step bound time ("score") on C4 against the default.  The probe
# builds' bounds are wrong by design; only the bound kernel's own HIP-event time is read.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("score", r["kernel_ms_per_step_isolated"]["score"], "knn", r["launch_ms"])'; }
for v in base pb1 pb2 base; do
  if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --steps 4 --iso-steps 4 --inflight 1 > $O/c4_$v.log 2>&1 || true
  echo "c4 $v $(show $O/c4_$v.log)"
done
