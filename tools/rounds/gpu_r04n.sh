# Round 4n: the multi-rank paths on the one GPU with gloo between the ranks (the whole N-rank path but
# RCCL): the reference's dataset run split round-robin over 2 ranks (detections all-gathered, parity vs
# the restatement's run over all 30 scenes), and the C4 global batch over 2 ranks; plus pytest -m gpu
# (the C++ host test's invalidate_models case).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 2 --config dataset --dist-backend gloo --cpu-sample 0 > $O/bench_dataset_gloo2.log 2>&1
tail -1 $O/bench_dataset_gloo2.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --cpu-sample 0 --steps 20 > $O/bench_c4_gloo2.log 2>&1
tail -1 $O/bench_c4_gloo2.log | cut -c1-200
