# Round 5t: LDS footprint for co-residency.  r05s: 3-tile distance stages (53.8 instead of 71.7 KiB per
# block) made the isolated launch 2 % slower but the pipelined C4 line ~2 % faster, a bound block (32 KiB)
# then fitting beside two distance blocks on a CU.  Variants (variants/libmim_<v>.so): distance stage
# st{2,3,4} x bound kernel LDS chunk bc{4,8} (bc4: 16 KiB per bound block); C4, C3 and the 32-problem
# shard, two interleaved rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "knn", r["launch_ms"], r["frac"], "score", r["kernel_ms_per_step_isolated"].get("score"))'; }
for i in 1 2; do
  for v in base st4bc4 st3bc8 st3bc4 st2bc4; do
    if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 --parity-sample 0 --iso-steps 4 > $O/s8_${v}_$i.log 2>&1; echo "s8 $v $(show $O/s8_${v}_$i.log)"
  done
done
