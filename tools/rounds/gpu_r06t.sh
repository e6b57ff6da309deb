# Round 6 t: issue rates of the mixed-precision count forms for the bound kernel (v_fma_mix*, v_dot2*,
# packed f16) next to v_fma_f32 -> profiles/r06t_issue_probe.txt
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/issue_probe tools/issue_probe.hip 2>/dev/null
PROBE_ONLY_A=1 timeout -k 10 120 /tmp/issue_probe > $O/issue_probe.txt 2>&1
cat $O/issue_probe.txt
