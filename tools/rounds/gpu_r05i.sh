# Round 5i: where the 32-problem shard (--shard-of 8) loses against the full batch: the same tree with the
# record gather left out (MIM_BENCH_GATHER=0, diagnostic), 16 / 24 batches in flight, and the whole-sweep
# distance schedule (MIM_KNN_TAIL=0); then the C4 kernel trace, HBM traffic and SQ counters (co-execution included).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "host", d["host_enqueue_ms_per_step"])'; }
timeout -k 10 120 ./tools/issue_probe > $O/issue_probe.txt 2>&1
for i in 1; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 > $O/s8_base_$i.log 2>&1; echo "base $(show $O/s8_base_$i.log)"
  MIM_BENCH_GATHER=0 timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 > $O/s8_nogather_$i.log 2>&1; echo "nogather $(show $O/s8_nogather_$i.log)"
  MIM_KNN_TAIL=0 timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 > $O/s8_notail_$i.log 2>&1; echo "notail $(show $O/s8_notail_$i.log)"
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --shard-of 8 --inflight 24 > $O/s8_if24_$i.log 2>&1; echo "inflight24 $(show $O/s8_if24_$i.log)"
done

timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/c4_base.log 2>&1; echo "c4 $(show $O/c4_base.log)"
MIM_BENCH_GATHER=0 timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/c4_nogather.log 2>&1; echo "c4 nogather $(show $O/c4_nogather.log)"
# kernel trace + HBM counters of C4 (tools/prof_round.sh), then SQ counters of the distance and bound
# kernels, the co-execution counter in a pass of its own
timeout -k 10 900 bash tools/prof_round.sh c4
K='knn2_i8|ransac_bound_mfma'
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d $O/pmc_sq$i -o run -- python3 bench.py --inflight 1 --steps 2 --warmup 1 --iso-steps 1 --cpu-sample 0 > $O/pmc_sq$i.log 2>&1 || echo "sq pass $i failed"
done
