# Round 6 ad: check kernel occupancy: 2 or 3 attempts per thread (cp2, cp3), register budget for 6 or 7 waves per SIMD (oc6, oc7) -> profiles/r06ad_check_occ_ab.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "chain", k.get("chain"), "check", k.get("check"), "parity", d["parity"]["checked"], d["parity"]["mismatch"])'; }
for i in 1 2; do
  for v in new cp2 cp3 oc6 oc7; do
    if [ $v = new ]; then L=""; else L=$V/libmim_$v.so; fi
    MIM_LIB=$L timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 10 > $O/${v}_$i.log 2>&1
    echo "$v run $i: $(show $O/${v}_$i.log)" | tee -a $O/summary.txt
  done
done
