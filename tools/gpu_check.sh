# quick GPU loop: parity tests + one bench line (each step under its own time limit)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -s -C oracle
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-problems ${CPU_PROBLEMS:-1} > gpurun_out/bench.log 2>&1
