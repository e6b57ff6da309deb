"""CPU-side checks of the C ABI: libmim.so builds for gfx950, loads, exports every include/mim.h symbol,
and reports a missing device loudly (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "mim.h")).read()
    return sorted(set(re.findall(r"\b(mim_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from computervision_objectdetection_featurematching_amd import build
    build.build()
    return ctypes.CDLL(build.SO)


def test_exports_every_declared_symbol(lib):
    syms = _header_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    from computervision_objectdetection_featurematching_amd import _lib
    assert sorted(_lib.EXPORTS) == syms


def test_version_and_params(lib):
    from computervision_objectdetection_featurematching_amd import _lib, default_params
    assert b"gfx950" in _lib.load().mim_version()
    p = default_params()
    assert p.ratio == pytest.approx(0.9) and p.min_good == 4 and p.min_inliers == 4
    assert p.ransac_thresh == 5.0 and p.max_iters == 2000 and p.confidence == 0.995
    assert p.det_lo == float(__import__("numpy").float32(0.1)) and p.det_hi == 10.0


def test_code_object_is_gfx950(lib):
    from computervision_objectdetection_featurematching_amd import build
    data = open(build.SO, "rb").read()
    assert b"gfx950" in data


def test_no_device_is_loud():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd._lib import MimError
    with pytest.raises(MimError):
        Matcher(0)


def test_struct_layouts():
    from computervision_objectdetection_featurematching_amd import _lib
    assert ctypes.sizeof(_lib.Params) == 56
    assert ctypes.sizeof(_lib.Result) == 96
    assert ctypes.sizeof(_lib.Problem) == 8


def test_cmake_drop_in_builds(tmp_path):
    """The CMake target the reference's pipeline links configures and builds the same
    library for gfx950, exporting every mim.h symbol."""
    import shutil
    import subprocess
    cmake = shutil.which("cmake")
    if cmake is None or not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("cmake / ROCm clang not available")
    b = tmp_path / "build"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    subprocess.run([cmake, "-S", ROOT, "-B", str(b), *gen, "-DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++",
                    "-DCMAKE_PREFIX_PATH=/opt/rocm"], check=True, capture_output=True, timeout=300)
    subprocess.run([cmake, "--build", str(b), "-j", "8"], check=True, capture_output=True, timeout=900)
    so = b / "libmim.so"
    assert so.exists() and b"gfx950" in so.read_bytes()
    lib = ctypes.CDLL(str(so))
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
