# Per-kernel SQ/TCC counters (separate --pmc passes, kernel trace only).
# usage: KREGEX='knn2_i8' PASSES='A B|C D' bash tools/prof_pmc_kernel.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck
K=${KREGEX:-ransac_bound}
PASSES=${PASSES:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES|SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS|SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM"}
i=0
IFS='|'
for C in $PASSES; do
  i=$((i+1))
  IFS=' '
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d gpurun_out/pmck/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > gpurun_out/pmck/p$i.log 2>&1
  IFS='|'
done
