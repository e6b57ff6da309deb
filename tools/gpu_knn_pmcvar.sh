# Distance-kernel variants: C3 bench line (isolated kNN ms) + two PMC passes on knn2_i8 each
# (effective clock = GRBM_GUI_ACTIVE / 8 / dispatch time; MFMA busy; wait/issue split).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pv
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  MIM_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 1 --cpu-sample 0 > gpurun_out/pv/$n.bench 2>&1 || { echo "$n bench failed"; tail -5 gpurun_out/pv/$n.bench; exit 1; }
  i=0
  for C in "$P1" "$P2"; do
    i=$((i+1))
    MIM_LIB=$PWD/$so timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex knn2_i8 \
      -d gpurun_out/pv/$n/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > gpurun_out/pv/$n.p$i.log 2>&1 || { echo "$n pmc $i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pv/$n > gpurun_out/pv/$n.summary.txt
  python3 - gpurun_out/pv/$n.bench gpurun_out/pv/$n.summary.txt <<'PY'
import json, re, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
c = {}
ms = None
for line in open(sys.argv[2]):
    m = re.match(r"mim::knn2_i8_kernel\s+(\S+)\s+total\s+(\S+)", line)
    if m: c[m.group(1)] = float(m.group(2))
    m = re.match(r"mim::knn2_i8_kernel\s+dispatch ms: (\S+)", line)
    if m: ms = float(m.group(1).rstrip(","))
clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e9 if ms else 0
cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / max(cyc, 1)
wc = c.get("SQ_WAVE_CYCLES", 1)
print(sys.argv[1].split("/")[-1], f"value {d['value']:.0f} iso_knn {r.get('isolated_kernel_ms_per_step', {}).get('knn')} "
      f"pmc_ms {ms} clk {clk:.2f}GHz mfma_util {util:.3f} wait {c.get('SQ_WAIT_ANY',0)/wc:.2f} "
      f"issue_stall {c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
      f"valu/mfma {c.get('SQ_INSTS_VALU',0)/max(c.get('SQ_INSTS_MFMA',1),1):.2f} salu/mfma {c.get('SQ_INSTS_SALU',0)/max(c.get('SQ_INSTS_MFMA',1),1):.2f}")
PY
done
