# variants bench + knn PMC passes on the default build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for so in computervision_objectdetection_featurematching_amd/lib/variants/libmim_*.so; do
  n=$(basename $so .so)
  MIM_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/var/$n.bench 2>&1
done
KREGEX=knn2_i8 PASSES="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU|SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS" bash tools/prof_pmc_kernel.sh
python3 tools/pmc_summary.py gpurun_out/pmck > gpurun_out/pmck/summary.txt
