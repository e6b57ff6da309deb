# Round 4r: the C++ drop-in path on the reference's images (tests/test_cpp_host.py: Detector::sift per model
# view, detect_scene_gray per scene, mim_detect.hpp boxes, against the restatement's golden outputs).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cpp_host.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_cpp.log 2>&1
tail -3 $O/pytest_cpp.log
