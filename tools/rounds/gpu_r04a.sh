# Round 4a: RCCL process group at N = 1 (bench default C4 through all_gather_into_tensor), the new
# GPU tests (C4 full batch over RCCL, SIFT limit paths), then C4 / c1img / dataset lines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config c1img > $O/bench_c1img.log 2>&1
tail -1 $O/bench_c1img.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config dataset --steps 3 > $O/bench_dataset.log 2>&1
tail -1 $O/bench_dataset.log | cut -c1-400
