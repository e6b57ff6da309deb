# parity tests, then the bench at 1..3 pipelined groups, with and without kernel timing
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -s -C oracle
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
for G in 1 2 3; do
  MIM_GROUPS=$G timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-problems 0 > gpurun_out/bench_g$G.log 2>&1
  MIM_GROUPS=$G timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-problems 0 --no-timing > gpurun_out/bench_nt_g$G.log 2>&1
done
