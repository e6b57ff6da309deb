set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > gpurun_out/prof2/log 2>&1
