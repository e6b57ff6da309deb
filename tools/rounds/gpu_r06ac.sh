# Round 6 ac: check kernel probes on C4 (isolated kernel times): the library (deferred attempts through
# their own kernel), pc1 (no deferred pass, so no fp32 'clear' test either), pc3 (every point gathered,
# a 16-add stand-in for the fp32 check), previous commit -> profiles/r06ac_check_probe.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  for v in new pc1 pc3 lds prev; do
    if [ $v = new ]; then L=""; else L=$V/libmim_$v.so; fi
    MIM_LIB=$L timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 10 > $O/${v}_$i.log 2>&1
    echo "$v run $i: $(show $O/${v}_$i.log)" | tee -a $O/summary.txt
  done
done
