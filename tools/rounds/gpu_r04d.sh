# Round 4d: sampler rework (attempt kernel marks repeated indices only, irr kernel resolves their
# redraw lengths, check kernel defers redraw / fp32-undecided attempts to a second pass): pytest -m gpu,
# C4 line, kernel trace of one isolated C4 batch.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --inflight 1 --steps 1 --warmup 0 --iso-steps 1 --cpu-sample 0 > $O/trace.log 2>&1
