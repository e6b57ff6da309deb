# Round 3w: distance-schedule parity test (MIM_KNN_SUB variants vs default, rows + records).
# -> gpurun_out/r03w/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -k "schedules or c5_dense" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -8 $O/pytest.log
