# Per-kernel SQ counters for the RANSAC kernels (separate --pmc passes, kernel trace only).
# usage: KREGEX='ransac_bound' bash tools/prof_pmc_kernel.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck
K=${KREGEX:-ransac_bound}
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d gpurun_out/pmck/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-problems 0 --no-timing > gpurun_out/pmck/p$i.log 2>&1
done
