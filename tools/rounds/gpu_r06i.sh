# r06i: SQ counters of the SIFT kernels (one standalone 640x480 call + the rest of time_sift --reps 1):
# wave lifetimes, instruction mix and waits of extrema / blur / orient / kp_post / descr, and
# GRBM_GUI_ACTIVE against the traced duration (the clock the kernels ran at).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
K='extrema_kernel|blur_reg|orient_kernel|kp_post|descr_kernel|refine_kernel'
i=0
for C in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "$K" \
     -d $O/p$i -o run -- python3 tools/time_sift.py --reps 1 > $O/p$i.log 2>&1 < /dev/null
done
echo done
