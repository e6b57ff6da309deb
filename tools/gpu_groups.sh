# bench at 1..3 pipelined groups (no kernel timing), each step under its own limit
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for G in 1 2 3; do
  MIM_GROUPS=$G timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-timing > gpurun_out/bench_nt_g$G.log 2>&1
done
