# Round 4s: the check kernel at higher occupancy (__launch_bounds__(256, 6 | 8): 80 / 64 VGPRs with 108 /
# 184 B of scratch spills, vs 91 VGPRs = 5 waves per SIMD now): same-box alternating C4 lines, 8 problems
# against the oracle each, isolated check-kernel times.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
lib() { case $1 in cur) unset MIM_LIB;; *) export MIM_LIB=$PWD/variants/libmim_$1.so;; esac; }
for rep in 1 2; do
  for v in cur occ6 occ8; do
    lib $v
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 8 > $O/c4_${v}_$rep.log 2>&1
    echo "c4 $v $(tail -1 $O/c4_${v}_$rep.log | cut -c95-150)"
  done
done
