# Round 5y3: SQ counters of the SIFT descriptor kernel (c1img, --inflight 1): which LDS counters gfx950
# offers, then two passes of SQ counters restricted to descr_kernel.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05y3
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*LDS[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT[A-Z_]*" $O/avail.txt | sort -u > $O/sq_names.txt || true
cat $O/sq_names.txt | tr '\n' ' '; echo
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex "descr_kernel" \
     -d $O/pmc$i -o run -- python3 bench.py --config c1img --steps 1 --warmup 1 --iso-steps 1 --cpu-sample 0 --parity-sample 0 --inflight 1 > $O/pmc$i.log 2>&1 || echo "pass $i failed"
done
