"""Build libmim.so in-tree for gfx950 (hipcc), the artefact that ships to the GPU box."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
SO = os.path.join(LIBDIR, "libmim.so")
SOURCES = ["knn.hip", "ransac.hip", "sift.hip", "api.cpp", "group.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: the RANSAC/DLT arithmetic must not be FMA-contracted (OpenCV's calib3d
# x86-64 build has no FMA), see DESIGN.md "Floating-point contract".
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-result", "-Wno-unused-function"]
# debug build (MIM_DEBUG=1): the in-kernel checks of csrc/mim_debug.h; extra defines for variant
# builds (tuning knobs of csrc/mim_internal.h, e.g. MIM_EXTRA_FLAGS=-DMIM_KNN_QT=4)
if os.environ.get("MIM_DEBUG") == "1":
    FLAGS.append("-DMIM_DEBUG")
FLAGS += os.environ.get("MIM_EXTRA_FLAGS", "").split()
# per-source flags: the RANSAC kernels are scalar fp32/fp64 code; v2f32 packing (v_pk_fma_f32 issues
# at half rate on gfx950 and needs SGPR-pair shuffles for uniform operands) only costs there; MFMA
# results in VGPRs (the bound kernel reads every accumulator with VALU ops, AGPRs would need a copy)
SRC_FLAGS = {"ransac.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]}


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def needs_build() -> bool:
    if not os.path.exists(SO):
        return True
    t = os.path.getmtime(SO)
    deps = sources() + [os.path.join(CSRC, "mim_internal.h"), os.path.join(CSRC, "mim_debug.h"),
                        os.path.join(HERE, "..", "include", "mim.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return SO
    os.makedirs(LIBDIR, exist_ok=True)
    # objects in a directory of this process's own and the library renamed into place, so processes
    # that build at the same time (the ranks of a multi-GPU bench) cannot mix each other's files
    import tempfile
    odir = os.environ.get("MIM_BUILD_DIR") or tempfile.mkdtemp(prefix="mim_build_")
    os.makedirs(odir, exist_ok=True)
    objs = []
    for src in sources():
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        cmd = [HIPCC, *FLAGS, *SRC_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        objs.append(obj)
    os.makedirs(os.path.dirname(os.path.abspath(SO)), exist_ok=True)
    tmp = f"{SO}.tmp{os.getpid()}"
    # librccl: the several-GPU group's all-gather (group.cpp)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs, "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    os.replace(tmp, SO)
    for o in objs:
        os.remove(o)
    if not os.environ.get("MIM_BUILD_DIR"):
        os.rmdir(odir)
    return SO


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(SO)
