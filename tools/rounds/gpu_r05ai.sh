# Round 5ai: the corpus failure of r05ah (near_line: filtered != all-exact with the LDS-staged prescreen):
# the corpus with the prescreen's exact recount (tools/diag_prescreen.py) on the LDS build and on the
# global-load build (variants/libmim_pglob.so), and with the prescreen off.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 300 python -u tools/diag_prescreen.py > $O/lds.log 2>&1 || true
grep -c "prescreen mismatch" $O/lds.log || true
grep "prescreen mismatch" $O/lds.log | head -8 || true
grep "differ:" $O/lds.log || tail -5 $O/lds.log
MIM_LIB=$PWD/variants/libmim_pglob.so timeout -k 10 300 python -u tools/diag_prescreen.py > $O/glob.log 2>&1 || true
grep -c "prescreen mismatch" $O/glob.log || true
grep "differ:" $O/glob.log || tail -5 $O/glob.log
MIM_PRESCREEN=0 timeout -k 10 300 python -u tools/diag_prescreen.py > $O/off.log 2>&1 || true
grep "differ:" $O/off.log || tail -5 $O/off.log
