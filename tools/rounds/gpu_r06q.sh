# r06q: blur tile heights: kernel traces of time_sift (cur: 32-row tiles; thb64: 64-row tiles for the
# half-widths 10 and 13; th16: 16-row tiles for all) -> the blur launches' durations.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
CUR=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
for v in cur thb64 th16; do
  L=$V/libmim_$v.so; [ $v = cur ] && L=$CUR
  MIM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- \
    python3 tools/time_sift.py --reps 5 > $O/trace_$v.log 2>&1 < /dev/null
done
echo done
