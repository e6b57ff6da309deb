# Round 6 y: where the check kernel's time goes: timing-only builds without the
# deferred pass (pc1) and also without the fp32 checkSubset (pc2; both give wrong samples), against the
# default library, C4 isolated kernel times -> profiles/r06y_check_probe.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "sample", k.get("sample"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 10 > $O/base_$i.log 2>&1
  echo "base run $i: $(show $O/base_$i.log)" | tee -a $O/summary.txt
  for v in pc1 pc2; do
    MIM_LIB=$PWD/$V/libmim_$v.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 10 > $O/${v}_$i.log 2>&1
    echo "$v run $i: $(show $O/${v}_$i.log)" | tee -a $O/summary.txt
  done
done
