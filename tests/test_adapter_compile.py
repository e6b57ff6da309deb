"""Compile-only check of the OpenCV drop-in (adapter/opencv/*.cpp) in this image, which has no OpenCV.

The adapter keeps the reference's signatures (/root/reference/include/TestsDetector.hpp:13-17,
ModelsDetector.hpp:13-14) and is built with the real OpenCV by CMake (-DMIM_WITH_OPENCV=ON).  Here it
is type-checked (`g++ -fsyntax-only`, nothing linked or run) against the reference's own headers and
tests/cv_stub — declarations of the few OpenCV names used, test infrastructure only — with and without
MIM_GPU_SIFT (SIFT and resize on the device).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INC = "/root/reference/include"


@pytest.mark.parametrize("src", ["TestsDetector.cpp", "ModelsDetector.cpp"])
@pytest.mark.parametrize("gpu_sift", [False, True])
def test_adapter_type_checks(src, gpu_sift):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    if not os.path.isdir(REF_INC):
        pytest.skip("the reference's headers are not here (GPU box)")
    if src == "ModelsDetector.cpp" and not gpu_sift:
        pytest.skip("without MIM_GPU_SIFT the reference's own ModelsDetector.cpp is built")
    cmd = ["g++", "-std=c++20", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "tests", "cv_stub"), "-I", REF_INC, "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "adapter", "opencv"), os.path.join(ROOT, "adapter", "opencv", src)]
    if gpu_sift:
        cmd.insert(1, "-DMIM_GPU_SIFT")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
