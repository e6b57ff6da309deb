# r06g: where the intermittent ~28 ms of a standalone sift_detect_compute call goes (r06e/r06f): host
# times of the call's phases (MIM_SIFT_TRACE=1: image copy enqueue, batch, fetch), four fresh processes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
for i in 1 2 3 4; do
  MIM_SIFT_TRACE=1 timeout -k 10 120 python3 -u tools/time_sift.py --reps 3 > $O/time_sift_cur_$i.log 2>&1
done
echo done
