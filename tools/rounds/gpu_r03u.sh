# Round 3u: refine phase times (shader cycles, s_memtime) of problem 0, MIM_REFINE_PROF build, C3 batch.
# -> gpurun_out/r03u/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
MIM_LIB=$PWD/$V/libmim_rprof.so timeout -k 10 300 python -u bench.py --config c3 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 --inflight 1 > $O/c3.log 2>&1
grep -c "refine-prof" $O/c3.log
grep "refine-prof" $O/c3.log | head -80
