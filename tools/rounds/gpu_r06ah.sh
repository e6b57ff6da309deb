# Round 6 ah: the attempt kernel loading the next round's draws while it reduces the current one
# (MIM_ATTEMPT_PREFETCH=1, variant apf) against the default, C4 isolated sampler times and lines
# -> profiles/r06ah_summary.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ah
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/base_$i.log 2>&1
  echo "base run $i: $(show $O/base_$i.log)" | tee -a $O/summary.txt
  MIM_LIB=$V/libmim_apf.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/apf_$i.log 2>&1
  echo "apf run $i: $(show $O/apf_$i.log)" | tee -a $O/summary.txt
done
