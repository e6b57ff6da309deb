# r06f: the standalone sift_detect_compute call (tools/time_sift.py) ran ~28 ms per 640x480 image in
# r06e on the current tree against 1.44 ms on HEAD's sift.hip while the batched scene path got faster:
# kernel + HIP runtime traces of time_sift for cur and prev, then time_sift x2 each again.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
CUR=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
for i in 1 2; do
  MIM_LIB=$CUR timeout -k 10 120 python3 -u tools/time_sift.py --reps 5 > $O/time_sift_cur_$i.log 2>&1
  MIM_LIB=$V/libmim_prev.so timeout -k 10 120 python3 -u tools/time_sift.py --reps 5 > $O/time_sift_prev_$i.log 2>&1
done
MIM_LIB=$CUR timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --output-format csv -d $O/cur -o run -- \
  python3 tools/time_sift.py --reps 3 > $O/trace_cur.log 2>&1 < /dev/null
MIM_LIB=$V/libmim_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prev -o run -- \
  python3 tools/time_sift.py --reps 3 > $O/trace_prev.log 2>&1 < /dev/null
echo done
