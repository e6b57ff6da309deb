# Round 3bo: the resize tests after the empty-destination case became an error check (was a skip)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03bo
timeout -k 10 300 python -u -m pytest tests/test_sift_gpu.py -q -k resize --timeout 120 --timeout-method thread > gpurun_out/r03bo/pytest.log 2>&1
tail -1 gpurun_out/r03bo/pytest.log
