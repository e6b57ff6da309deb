# Round 6 ai: check kernel attempts per thread on the round-6 fp32 checkSubset (77 registers at 4 per
# thread): 2 (cp2, 62 registers: 8 waves per SIMD) and 3 (cp3) against the default, C4 isolated times
# -> profiles/r06ai_summary.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ai
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  for v in base cp2 cp3; do
    if [ $v = base ]; then L=""; else L=$V/libmim_$v.so; fi
    MIM_LIB=$L timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/${v}_$i.log 2>&1
    echo "$v run $i: $(show $O/${v}_$i.log)" | tee -a $O/summary.txt
  done
done
